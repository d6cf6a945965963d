"""Runtime flags (environment variables): the ONE place xdot reads ``XDOT_*`` variables.

Read once at import (``FLAGS.reload()`` re-reads them) and overridable in code; the native
extension reads the ones marked (C++) itself, at its first use.  The reference has a single
flag (``DISTRIBUTED_DOT_DEBUG``, ``multiplication/functions.py:21``); everything else here is a
documented default of this MI355X build, mostly with the measurement that chose it.

==========================  ========  ===========================================================
variable                    default   effect
==========================  ========  ===========================================================
``XDOT_DEBUG`` /            0         print per-op shapes, HBM delta and synced time (reference
``DISTRIBUTED_DOT_DEBUG``             alias)
``XDOT_CHECK``              0         all-gather an op fingerprint before every distributed op and
                                      raise on rank divergence instead of hanging  [collective]
``XDOT_BACKEND``            auto      ``auto`` | ``hip`` | ``torch``: compute backend of GPU tensors
``XDOT_ALLOW_TORCH_FALLBACK`` 0       let GPU ops fall back to torch when ``_C.so`` is absent
                                      (default: fail loudly)
``XDOT_EXT_PATH``           (in-tree) load this build of the extension instead of ``xdot/_C.so``
                                      (skips the build-id check)
``XDOT_AUTO_REBUILD``       1         an in-tree ``_C.so`` whose embedded build id differs from the
                                      ``csrc/`` tree is rebuilt on load (0: raise instead)
``XDOT_COMM_TIMEOUT_S``     600       bound of every collective (process group timeout; also the
                                      default bound of the IPC kernels' device-side waits)
``XDOT_CHUNK_BUDGET_MB``    0 (auto)  transient-buffer budget of the chunk planner and of the
                                      grouped offset gathers of ``nt`` / ``all``  [collective]
``XDOT_OPS_SCHEDULE``       gather    ``ring``: the distributed products move shards rank to rank
                                      (send/recv) instead of all-gather / reduce-scatter  [collective]
``XDOT_GATHER_CHUNKS``      0 (auto)  row chunks of the fused attention's gather / reduce-scatter
                                      pipeline (auto: 2 from 8 ranks on, else 1;
                                      profiles/r2_gather_chunks.md)  [collective]
``XDOT_LOCAL_FIRST``        1         fused forward: the rank's own block runs under the gather
                                      (0: wait for the whole gather)  [collective]
``XDOT_GRAD_FP32``          0         reduce-scatter the gathered-side gradient partials in fp32
                                      (default: rounded once to bf16/fp16 in the kernel)  [collective]
``XDOT_GRAD_WIRE32``        1         fused node hands 16-bit weight gradients to GradSync(reduce_dtype=
                                      fp32) in fp32, straight from the kernels' sums (0: in the
                                      parameter dtype, converted before the all-reduce)  [collective]
``XDOT_IPC``                0         all-gathers / reduce-scatters as native xGMI pull kernels over
                                      HIP IPC (``csrc/ipc.hip``)  [collective]
``XDOT_IPC_MB``             512       IPC staging MiB per slot (routes IPC vs RCCL by size)  [collective]
``XDOT_IPC_WGS``            64        workgroups (byte ranges) per IPC collective
``XDOT_IPC_TIMEOUT_S``      (comm)    bound of every IPC device-side wait
``XDOT_PRESCALE``           1         pre-multiply the row side by scale·log2 e once per forward
                                      (seeded score accumulators; forward 2.11 -> 1.98 ms)
``XDOT_FP32_MODE``          exact     fp32 flash kernels and fp32 GEMMs (read by Python only, per
                                      call; passed to the kernels): ``exact`` (fp32 MFMA, ~5e-7
                                      relative vs fp64: the reference's precision) or ``split``
                                      (opt-in, like TF32: hi/lo bf16 halves, 3 bf16 products:
                                      <= 9e-6 flash, <= 2e-5 GEMM; profiles/r3_fp32_split.md)
``XDOT_FP32_SCORES``        1         fp32 flash (exact and split): the forward stores the raw scores and the
                                      backward reads S / dS instead of recomputing them (6 fp32
                                      products per step instead of 9; needs R*T*H*4 bytes)
``XDOT_FP32_SCORES_FRAC``   0.5       ... only when that fits this fraction of the free device memory
``XDOT_FP32_SCORES_DS``     1         ... and a second buffer for dS when both fit: the column side's
                                      dV pass then runs concurrently with the row kernel
``XDOT_F32_FUSED_COLS``      1         exact fp32, D <= 128: the column side as ONE fused pass (dP, dQ, dV per
                                      tile; S overwritten with dS in place, one score buffer) instead
                                      of a dQ pass and a dV pass (step 51.5-51.9 -> 50.1 ms, one box;
                                      profiles/r6_fp32.md)
``XDOT_FP32_DS_ONLY``       split     fp32 families that keep only the dS buffer (the forward stores
                                      nothing, the single-pass column kernel recomputes S and stores
                                      dS, the row kernel reads it: 40 GB of score traffic per step
                                      instead of 100): ``split`` (the memory-bound split-bf16
                                      family), ``all``, ``none``
``XDOT_FUSED_MODULE``       1         the module's flash path as ONE autograd node (projections +
                                      attention + output projection, xdot/models/fused.py; 0: one
                                      node per op)
``XDOT_MASK_ASYNC``         0         pack the attention mask on a side stream (neutral at N=1,
                                      1.7 % slower at the N=8 rank: profiles/r1_s7_mask_async_ab.md)
``XDOT_WGRAD_SIDE``         0         weight gradients on side streams beside the attention
                                      backward (same GPU time, +0.1-0.4 ms host per step: off;
                                      profiles/r4_s2.md)
``XDOT_INLINE_BACKWARD``    1         xdot.ops.loss.backward runs the backward on the calling thread
                                      (no autograd worker-thread hand-off: -0.2 ms host per step)
``XDOT_WGRAD``              1         Linear weight gradients on csrc/gemm_wgrad.hip (0: gemm3 split-K)
``XDOT_WGRAD_PAIR``         1         the fused backward's dWk and dW[q|v] in one launch (A/B knob)
``XDOT_ROWS_SPLIT``         0         column splits of the fused backward's row-side kernel (0: the
                                      launcher's occupancy model; A/B knob)
``XDOT_F32_PROJ``           1         exact-fp32 projections / weight gradients on the exact-fp32 GEMM kernels (both fp32 modes)
                                      (0: the library's fp32 GEMM)
``XDOT_PROJ``               1         projection forward / input gradient on csrc/gemm_proj.hip
                                      (1 / 2: every eligible shape, the 25000-row N=1 products
                                      included since round 6; 0: library)
``XDOT_RING_OVERLAP``       auto      ring attention backward on two streams (auto: >= 1024 row
                                      tiles of 128 x heads)
``XDOT_RING_BIDIR``         1         ring attention: half of every block each way round the ring
                                      (two xGMI links per hop), 16-bit accumulators  [collective]
``XDOT_ROCTX`` (C++)        0         roctx ranges around every native op (rocprofv3 markers)
``XDOT_GEMM_LIB`` (C++)     0         which plain large products may run on the library GEMM
                                      (hipBLASLt, ``csrc/bindings.cpp``): unset / 0 = none (every
                                      product on the xdot kernels: exact fp32 on csrc/gemm2_f32.hip
                                      / gemm_f32.hip), ``fp32`` = exact-fp32 ones (the round-4
                                      default, kept for A/B), 1 = 16-bit ones too
``XDOT_GEMM3`` (C++)        1         16-bit products with M, N >= 256 and beta = 0 run the 8-phase
                                      16x16x32 kernel (``csrc/gemm3.hip``; 0: the 256x256 v2 kernel)
``XDOT_CSPLIT`` (C++)        auto      row splits of the fp32 column kernels against the last-round
                                      tail (fp32 partials, ordered sum; auto: occupancy round
                                      model; n: n splits <= 4, also for the 16-bit pipelined kernel,
                                      whose auto is 1)
``XDOT_F32_SPLIT`` (C++)     auto      column splits of the fp32 forward / row-side kernels: auto =
                                      occupancy round model of the fp32 instantiation (up to 8);
                                      fwd = forward only; old = the 16-bit model; n = forced
``XDOT_F32_FWD_DIRECT`` (C++) 1        the score-storing exact-fp32 forward scatters S straight to the
                                      buffer (no LDS transpose tile: three workgroups per CU at
                                      D <= 96); 0 = the LDS-transposed store at two per CU
``XDOT_WIDE_SPLIT`` (C++)    auto      split counts of the wide-head (D > 128) kernels from their own
                                      occupancy (row splits of both column passes, column splits
                                      of forward / row side); 0 = previous model; n = forced
``XDOT_HIPCC_FLAGS`` (build)          extra hipcc flags for ``python -m xdot.build``
==========================  ========  ===========================================================

Variables marked [collective] change how many collectives an op issues (or their dtype):
ranks that disagree would hang, so :func:`collective_knobs` is cross-checked by
``xdot.utils.comm.init`` when it creates a multi-rank communicator.
"""
from __future__ import annotations

import os


def _flag(*names: str, default: str = "0") -> bool:
    for n in names:
        v = os.environ.get(n)
        if v is not None:
            return v.strip().lower() not in ("", "0", "false", "no", "off")
    return default not in ("0", "")


def _str(name: str, default: str) -> str:
    return (os.environ.get(name, default) or default).strip().lower()


def _num(name: str, default, typ=float):
    v = os.environ.get(name)
    if v is None or not v.strip():
        return default
    return typ(v)


class _Flags:
    def __init__(self):
        self.reload()

    def reload(self):
        self.debug = _flag("XDOT_DEBUG", "DISTRIBUTED_DOT_DEBUG")
        self.check = _flag("XDOT_CHECK")
        self.backend = _str("XDOT_BACKEND", "auto")
        self.allow_torch_fallback = _flag("XDOT_ALLOW_TORCH_FALLBACK")
        self.ext_path = os.environ.get("XDOT_EXT_PATH") or None
        self.auto_rebuild = _flag("XDOT_AUTO_REBUILD", default="1")
        self.comm_timeout_s = _num("XDOT_COMM_TIMEOUT_S", 600.0)
        self.chunk_budget_mb = _num("XDOT_CHUNK_BUDGET_MB", 0.0)
        self.ops_schedule = _str("XDOT_OPS_SCHEDULE", "gather")
        self.gather_chunks = _num("XDOT_GATHER_CHUNKS", 0, int)  # 0: auto
        self.local_first = _flag("XDOT_LOCAL_FIRST", default="1")
        self.grad_fp32 = _flag("XDOT_GRAD_FP32")
        self.grad_wire32 = _flag("XDOT_GRAD_WIRE32", default="1")
        self.ipc = _flag("XDOT_IPC")
        self.ipc_mb = _num("XDOT_IPC_MB", 512.0)
        self.ipc_wgs = _num("XDOT_IPC_WGS", 64, int)
        self.ipc_timeout_s = _num("XDOT_IPC_TIMEOUT_S", self.comm_timeout_s)
        self.prescale = _flag("XDOT_PRESCALE", default="1")
        self.fp32_mode = _str("XDOT_FP32_MODE", "exact")
        self.mask_async = _flag("XDOT_MASK_ASYNC")
        self.fp32_scores = _flag("XDOT_FP32_SCORES", default="1")
        self.fp32_scores_frac = _num("XDOT_FP32_SCORES_FRAC", 0.5)
        self.fp32_scores_dsbuf = _flag("XDOT_FP32_SCORES_DS", default="1")
        self.f32_fused_cols = _flag("XDOT_F32_FUSED_COLS", default="1")
        self.fp32_ds_only = _str("XDOT_FP32_DS_ONLY", "split")
        self.fused_module = _flag("XDOT_FUSED_MODULE", default="1")
        self.wgrad_side = _flag("XDOT_WGRAD_SIDE", default="0")
        self.proj_kernel = _num("XDOT_PROJ", 1, int)
        self.f32_proj = _flag("XDOT_F32_PROJ", default="1")
        self.inline_backward = _flag("XDOT_INLINE_BACKWARD", default="1")
        self.rows_split = _num("XDOT_ROWS_SPLIT", 0, int)
        self.wgrad_kernel = _flag("XDOT_WGRAD", default="1")
        self.wgrad_pair = _flag("XDOT_WGRAD_PAIR", default="1")
        self.ring_overlap = _str("XDOT_RING_OVERLAP", "auto")
        self.ring_bidir = _flag("XDOT_RING_BIDIR", default="1")
        self.hipcc_flags = os.environ.get("XDOT_HIPCC_FLAGS")


FLAGS = _Flags()

# flags that change the number (or dtype) of the collectives an op issues
COLLECTIVE_KNOBS = ("check", "chunk_budget_mb", "ops_schedule", "gather_chunks", "local_first", "grad_fp32", "grad_wire32",
                    "ipc", "ipc_mb", "ipc_wgs", "ring_bidir")


def collective_knobs() -> dict:
    """This process's values of the [collective] flags (every rank must agree on them)."""
    return {k: getattr(FLAGS, k) for k in COLLECTIVE_KNOBS}
