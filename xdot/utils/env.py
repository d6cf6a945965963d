"""Runtime flags (environment variables), read once at import and overridable in code.

=============================  ==========================================================
``XDOT_DEBUG`` / ``DISTRIBUTED_DOT_DEBUG``  print per-op shapes, HBM delta and synced time
                                           (reference alias: ``functions.py:21``)
``XDOT_CHECK``                 all-gather an op fingerprint before every distributed op
                               and raise on rank divergence (instead of hanging)
``XDOT_BACKEND``               ``auto`` | ``hip`` | ``torch``: compute backend for GPU tensors
``XDOT_ALLOW_TORCH_FALLBACK``  ``1`` lets GPU ops fall back to torch when ``_C.so`` is absent
                               (default: fail loudly)
``XDOT_COMM_TIMEOUT_S``        collective timeout in seconds (default 600)
``XDOT_CHUNK_BUDGET_MB``       transient-buffer budget used by the chunk planner (``offset='auto'``)
                               and by the grouped offset-row gathers of ``nt`` / ``all`` (a
                               quarter per group; default 256 MB per group)
``XDOT_GRAD_FP32``             ``1``: the fused attention's gathered-side gradient partials are
                               kept and reduce-scattered in fp32 (default: rounded once to
                               the bf16/fp16 compute dtype in the kernel, half the bytes)
``XDOT_ROCTX``                 ``1``: roctx ranges around every native op (rocprofv3 markers)
``XDOT_GATHER_CHUNKS``         row chunks of the fused attention's all-gather / reduce-scatter
                               pipeline with several ranks (default auto: 2 from 8 ranks on, else
                               1; with a 300 GB/s link model 2 chunks save 44 µs per N=8 rank step
                               and lose 12 µs at N=4, profiles/r2_gather_chunks.md)
``XDOT_LOCAL_FIRST``           ``0``: with several ranks the fused forward waits for the whole
                               all-gather, then runs one kernel over all T columns (default 1:
                               the rank's own block runs first, under the gather, then the peer
                               blocks of each chunk as it lands; one log-sum-exp combine)
``XDOT_MASK_ASYNC``            ``1``: pack the attention mask on a side stream, overlapping the
                               projection GEMMs (default off: neutral at N=1, 1.7 % slower at the
                               emulated N=8 rank, profiles/r1_s7_mask_async_ab.md; with several
                               ranks packing already overlaps the all-gather)
``XDOT_PRESCALE``              ``0``: flash kernels scale every score by scale*log2 e (default 1:
                               the row side is pre-multiplied once per forward — one bf16
                               rounding, the same buffer for forward and backward — and the
                               score accumulators are seeded with the row max / LSE; forward
                               2.11 -> 1.98 ms at T=R=25000)
``XDOT_RING_OVERLAP``          ring attention backward: ``1`` runs each block's gathered-side and
                               row-side kernels on two streams, ``0`` on one; default ``auto``:
                               two streams when a block has >= 1024 row tiles of 128 x heads
                               (measured, 1x MI355X, T=25000: N=1 9.21 -> 8.71 ms with two
                               streams, emulated N=8 rank 2.46 -> 2.63 ms, i.e. worse)
``XDOT_BWD_OVERLAP``           fused attention backward: ``1`` runs the row-side kernel concurrently
                               with the gathered-side kernel (two streams), ``0`` after it (the
                               reduce-scatter still overlaps it); default ``auto``: concurrent
                               when the rank has >= XDOT_BWD_OVERLAP_TILES row tiles of 128 x heads
                               (default 0: always; back to back measured slower at every rank
                               shape, profiles/r2_bwd_overlap.md)
``XDOT_BWD_SIDE_PRIO``         priority of the fused backward's gathered-side stream (default -1 =
                               high; 0 measured slower at N=1 and N=8, profiles/r2_bwd_overlap.md)
``XDOT_WGRAD_PATH``            weight-gradient GEMM: ``auto`` (the 256x256 split-K kernel) or ``128``
                               (K slabs of the 128x128 kernel, ``XDOT_WGRAD_SPLITS`` slabs);
                               profiles/r2_wgrad_route.md
``XDOT_ROWS_PIPE``             ``0``: plain (not software-pipelined) body of the flash backward
                               row kernel (default 1: VALU of one sub-tile issues between the
                               next sub-tile's MFMAs; 1.5 % faster kernel)
``XDOT_ROWS_NSPLIT``           column splits of the flash backward row kernel (default: the
                               occupancy model; 1 measured 7 % / 32 % slower at N = 1 / 8 ranks)
``XDOT_OPS_SCHEDULE``          ``ring``: the distributed products (``nt`` / ``all`` / ``tn`` and the
                               autograd ops / materialised path built on them) move the shards
                               rank to rank over point-to-point send/recv instead of all-gather /
                               reduce-scatter (default ``gather``: faster over xGMI's full mesh;
                               the ring holds two shards instead of the gathered side)
``XDOT_IPC``                   ``1``: with RCCL and several ranks, all-gathers and reduce-scatters
                               run as native xGMI pull kernels over HIP IPC
                               (``xdot/utils/ipc.py``, ``csrc/ipc.hip``; default 0 = RCCL).
                               ``XDOT_IPC_MB`` staging MiB per slot (512), ``XDOT_IPC_TIMEOUT_S``
                               bound of every device-side wait (30),
                               ``XDOT_IPC_WGS`` workgroups (byte ranges) per collective (128)
``XDOT_WGRAD_SIDE``            ``0``: the packed [q|v] projection's weight gradient runs on the
                               main stream after the attention backward (default 1: on the
                               backward's priority stream as soon as the gathered-side gradient
                               lands, overlapping the row-side kernel)
``XDOT_EXT_PATH``              load this build of the extension instead of ``xdot/_C.so``
=============================  ==========================================================
"""
from __future__ import annotations

import os


def _flag(*names: str, default: str = "0") -> bool:
    for n in names:
        v = os.environ.get(n)
        if v is not None:
            return v.strip().lower() not in ("", "0", "false", "no", "off")
    return default not in ("0", "")


class _Flags:
    def __init__(self):
        self.reload()

    def reload(self):
        self.debug = _flag("XDOT_DEBUG", "DISTRIBUTED_DOT_DEBUG")
        self.check = _flag("XDOT_CHECK")
        self.backend = os.environ.get("XDOT_BACKEND", "auto").lower()
        self.allow_torch_fallback = _flag("XDOT_ALLOW_TORCH_FALLBACK")
        self.chunk_budget_mb = float(os.environ.get("XDOT_CHUNK_BUDGET_MB", "0") or 0)
        self.grad_fp32 = _flag("XDOT_GRAD_FP32")
        self.gather_chunks = int(os.environ.get("XDOT_GATHER_CHUNKS", "0") or 0)  # 0: auto
        self.mask_async = _flag("XDOT_MASK_ASYNC")
        self.wgrad_side = _flag("XDOT_WGRAD_SIDE", default="1")
        self.local_first = _flag("XDOT_LOCAL_FIRST", default="1")
        self.prescale = _flag("XDOT_PRESCALE", default="1")
        self.ring_overlap = os.environ.get("XDOT_RING_OVERLAP", "auto").strip().lower() or "auto"
        self.bwd_overlap = os.environ.get("XDOT_BWD_OVERLAP", "auto").strip().lower() or "auto"
        self.ops_schedule = os.environ.get("XDOT_OPS_SCHEDULE", "gather").strip().lower() or "gather"


FLAGS = _Flags()
