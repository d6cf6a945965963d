"""Python face of the flash-attention kernels (``csrc/flash_fwd.hip``, ``csrc/flash_bwd.hip``,
``csrc/mask_pack.hip``).

Tensors are head-interleaved: ``rows`` (B, R, H*D) local query-side rows, ``kc``/``vc``
(B, T, H*D) the gathered key/value side.  The RCCL all-gather produces rank-major
(N, B, Rc, H*D); :func:`gathered_to_btc` turns that into (B, T, H*D) (a free view for B = 1)
and :func:`btc_to_rank_major` maps the fp32 key/value-side gradients back for the
reduce-scatter.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import _ext
from ..utils.env import FLAGS


class PackedMask:
    """Boolean (B, R, T) mask compressed to per-row bit words ``bits`` (B, ceil(T/64), R),
    the same bits column-major per 64-row tile ``bits_t`` (B, ceil(R/64), Tpad) for the
    backward column kernel, and per (32-row, 64-col) tile ``flags`` (0 none / 1 all / 2 some
    masked)."""

    __slots__ = ("bits", "flags", "bits_t", "shape")

    def __init__(self, bits: torch.Tensor, flags: torch.Tensor, bits_t: torch.Tensor, shape):
        self.bits, self.flags, self.bits_t, self.shape = bits, flags, bits_t, tuple(shape)

    @property
    def nothing_masked(self) -> bool:  # host sync; diagnostics only
        return bool((self.flags == 0).all())


def prepare_mask(mask: Optional[torch.Tensor], B: int, R: int, T: int) -> Optional[PackedMask]:
    if mask is None:
        return None
    if tuple(mask.shape) != (B, R, T):
        raise ValueError(f"mask must be (B, R, T) = {(B, R, T)}, got {tuple(mask.shape)}")
    bits, flags, bits_t = _ext.ops().mask_pack(mask.to(torch.bool).contiguous())
    return PackedMask(bits, flags, bits_t, mask.shape)


class _MaskEntry:
    __slots__ = ("ref", "version", "packed", "none_ev", "none_host")


class MaskCache:
    """Packed masks keyed on the boolean tensor that produced them.

    A training loop passes the same mask object every step (the reference's ``example.py``
    builds it once); re-packing it costs a full read of the (B, R, T) bool tensor per step
    (625 MB at T = 25000, N = 1).  An entry is valid while the tensor is alive (a weak
    reference whose finaliser evicts the entry, so a new tensor at a recycled address never
    hits) and its ``_version`` — bumped by every in-place write — is unchanged.

    All-False short-circuit: when a mask is packed, "any tile masked?" is copied to pinned host
    memory without a sync; on a later hit whose copy has landed and reads False, the cache
    hands out ``None`` (the kernels' no-mask path, nothing to stage per tile)."""

    def __init__(self, capacity: int = 8):
        self.capacity = capacity
        self._d = {}

    def _evict(self, key):
        self._d.pop(key, None)

    def get(self, mask: torch.Tensor, tag, pack):
        """``pack()`` -> PackedMask on a miss; ``tag`` distinguishes views packed from the
        same tensor (row chunks)."""
        import weakref

        key = (id(mask), tag)
        e = self._d.get(key)
        if e is not None and e.ref() is mask and e.version == mask._version:
            if e.none_ev is not None and e.none_ev.query():
                if not bool(e.none_host.item()):
                    return None
                e.none_ev = None
            return e.packed
        packed = pack()
        if packed is None:
            return None
        e = _MaskEntry()
        e.ref = weakref.ref(mask, lambda _r, k=key, c=self: c._evict(k))
        e.version = mask._version
        e.packed = packed
        e.none_ev, e.none_host = None, None
        if packed.flags.is_cuda:
            e.none_host = torch.empty((), dtype=torch.bool, pin_memory=True)
            # the flag rows are padded to a multiple of 4 tiles with 1 ("all masked"): only the
            # ceil(T/64) real column tiles count
            nkt = (packed.shape[-1] + 63) // 64
            e.none_host.copy_(packed.flags[..., :nkt].any(), non_blocking=True)
            e.none_ev = torch.cuda.Event()
            e.none_ev.record()
        if len(self._d) >= self.capacity:
            self._d.pop(next(iter(self._d)))
        self._d[key] = e
        return packed

    def clear(self):
        self._d.clear()


MASK_CACHE = MaskCache()


def prepare_mask_cached(mask: Optional[torch.Tensor], B: int, R: int, T: int, tag=None,
                        view=None) -> Optional[PackedMask]:
    """:func:`prepare_mask` through :data:`MASK_CACHE` (``view(mask)``: the slice to pack)."""
    if mask is None:
        return None
    return MASK_CACHE.get(mask, tag, lambda: prepare_mask(mask if view is None else view(mask), B, R, T))


class PendingMask:
    """A mask being packed on a side stream (:func:`prepare_mask_async`): the packing overlaps
    whatever the current stream does meanwhile (the projection GEMMs); :meth:`get` orders the
    calling stream after it."""

    __slots__ = ("raw", "shape", "_packed", "_event")

    def __init__(self, raw: torch.Tensor, packed: PackedMask, event):
        self.raw, self.shape, self._packed, self._event = raw, tuple(raw.shape), packed, event

    def get(self) -> Optional[PackedMask]:
        cur = torch.cuda.current_stream(self.raw.device)
        cur.wait_event(self._event)
        if self._packed is None:  # cached all-False mask
            return None
        for t in (self._packed.bits, self._packed.flags, self._packed.bits_t):
            t.record_stream(cur)
        return self._packed


_AUX = {}


def prepare_mask_async(mask: torch.Tensor, B: int, R: int, T: int) -> PendingMask:
    """:func:`prepare_mask` on a per-device side stream, ordered after the current stream."""
    dev = mask.device
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _AUX:
        _AUX[i] = torch.cuda.Stream(device=i)
    side = _AUX[i]
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        packed = prepare_mask_cached(mask, B, R, T)
        ev = torch.cuda.Event()
        ev.record(side)
    mask.record_stream(side)
    return PendingMask(mask, packed, ev)


def gathered_to_btc(g: torch.Tensor) -> torch.Tensor:
    """(N, B, Rc, C) rank-major all-gather output -> (B, N*Rc, C)."""
    N, B, Rc, C = g.shape
    if B == 1:
        return g.view(1, N * Rc, C)
    return g.permute(1, 0, 2, 3).reshape(B, N * Rc, C)


def btc_to_rank_major(x: torch.Tensor, N: int) -> torch.Tensor:
    """(B, T, C) -> (N, B, T/N, C) contiguous (reduce-scatter send layout)."""
    B, T, C = x.shape
    if B == 1:
        return x.view(N, 1, T // N, C)
    return x.view(B, N, T // N, C).permute(1, 0, 2, 3).contiguous()


def _kv(x: torch.Tensor) -> torch.Tensor:
    """key/value-side operand: (B, T, C) with unit inner stride (row stride may exceed C)."""
    if x.dim() == 3 and x.stride(-1) == 1 and x.stride(1) % 8 == 0 and (x.shape[0] == 1 or x.stride(0) == x.shape[1] * x.stride(1)):
        return x
    return x.contiguous()


def _mask_args(mk: Optional[PackedMask]):
    return (mk.bits, mk.flags) if mk is not None else (None, None)


def prescale(rows: torch.Tensor, scale: float) -> torch.Tensor:
    """``rows * (scale * log2 e)`` in the input dtype (one rounding), the form the kernels take with
    ``prescaled=True``: their score accumulators are then seeded with the row max / LSE and the
    probabilities are ``2^acc`` with no per-score FMA.  Forward and backward must see the SAME
    pre-scaled buffer."""
    return _ext.ops().flash_prescale(rows.contiguous(), float(scale))


FP32_MODES = {"exact": 0, "split": 1}


def fp32_code(dtype: torch.dtype, mode: Optional[str] = None) -> int:
    """Kernel family of fp32 operands: 0 exact fp32 (``csrc/flash_f32.hip``, the default: ~5e-7
    relative error vs fp64, the reference's precision), 1 split-bf16 (``csrc/flash_x3.hip``,
    opt-in: 3 bf16 MFMAs per product, <= 9e-6; profiles/r3_fp32_split.md).  ``mode`` None: ``XDOT_FP32_MODE``.  0 for 16-bit dtypes."""
    if dtype != torch.float32:
        return 0
    mode = FLAGS.fp32_mode if mode is None else mode
    if mode not in FP32_MODES:
        raise ValueError(f"fp32 mode must be one of {sorted(FP32_MODES)}, got {mode!r}")
    return FP32_MODES[mode]


def score_buffer_numel(B: int, H: int, R: int, T: int) -> int:
    """Floats of the fp32 score buffer: (B*H, ceil(R/32), ceil(T/32)) blocks of 32x32, plus one
    dump block the waves that own no block (rows past R, columns past T) write into."""
    return (B * H * ((R + 31) // 32) * ((T + 31) // 32) + 1) * 1024


def score_buffer(B: int, H: int, R: int, T: int, device) -> Optional[torch.Tensor]:
    """The fp32 score buffer (``csrc/flash_f32.hip`` exact, ``csrc/flash_x3.hip`` split; score-buffer mode) or None.

    The forward stores every computed score tile there; the backward's column kernel reads S
    instead of recomputing it and overwrites it with dS, which the row kernel reads: 6 fp32
    products per step instead of 9 for 8 bytes of otherwise idle HBM traffic per score.  It is
    R x T x H floats (20 GB at T = R = 25000, H = 8), so it is only taken when it fits within
    ``XDOT_FP32_SCORES_FRAC`` of the memory free on the device (free + cached by torch); else
    None and the kernels recompute (``XDOT_FP32_SCORES=0`` forces that)."""
    if not FLAGS.fp32_scores:
        return None
    n = score_buffer_numel(B, H, R, T)
    dev = torch.device(device)
    free, _ = torch.cuda.mem_get_info(dev)
    cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    if 4 * n > FLAGS.fp32_scores_frac * (free + cached):
        return None
    return torch.empty(n, dtype=torch.float32, device=dev)


def fused_cols_wanted(fp32_mode: int, D: int) -> bool:
    """The exact-fp32 backward's column side as ONE fused pass (dP, dQ and dV per tile, S
    overwritten with dS in place; ``XDOT_F32_FUSED_COLS``) instead of a dQ pass and a dV pass:
    exact family, D <= 128."""
    return FLAGS.f32_fused_cols and fp32_mode == 0 and D <= 128


def score_buffers(B: int, H: int, R: int, T: int, device, dsbuf: bool = True):
    """(S buffer, dS buffer) for the backward's concurrent schedule, (S buffer, None) for the
    in-place one, or None (recompute): like :func:`score_buffer`, the dS buffer only when both fit
    within ``XDOT_FP32_SCORES_FRAC`` of the free device memory.  With a separate dS buffer the
    column side runs its dQ pass first (S -> dS), then its dV pass (reads S) CONCURRENTLY with the
    row kernel (reads dS): two one-product kernels side by side instead of back to back.
    ``dsbuf=False``: the S buffer only (in place)."""
    if not FLAGS.fp32_scores:
        return None
    n = score_buffer_numel(B, H, R, T)
    dev = torch.device(device)
    free, _ = torch.cuda.mem_get_info(dev)
    cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    room = FLAGS.fp32_scores_frac * (free + cached)
    if 8 * n <= room and FLAGS.fp32_scores_dsbuf and dsbuf:
        both = torch.empty(2 * n, dtype=torch.float32, device=dev)
        return both[:n], both[n:]
    if 4 * n <= room:
        return torch.empty(n, dtype=torch.float32, device=dev), None
    return None


def ds_only_wanted(fp32_mode: int, D: int) -> bool:
    """Whether fp32 family ``fp32_mode`` (0 exact, 1 split) at head dim ``D`` keeps only a dS
    buffer (``XDOT_FP32_DS_ONLY``): the forward stores nothing, the single-pass column kernel
    recomputes S and stores dS, the row kernel reads dS.  The split family's kernels are bound by
    the score traffic (S written, read twice, dS written and read: 100 GB per step at T = R =
    25000, H = 8); this mode moves 40 GB for one recomputed product on the column side."""
    if D > 128:
        return False
    m = FLAGS.fp32_ds_only
    return m == "all" or (m == "split" and fp32_mode == 1)


def ds_buffer(B: int, H: int, R: int, T: int, device) -> Optional[torch.Tensor]:
    """The dS buffer of the dS-only mode (:func:`ds_only_wanted`), same size rule as
    :func:`score_buffer`, or None."""
    return score_buffer(B, H, R, T, device)


def fwd(rows: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, mk: Optional[PackedMask], H: int,
        scale: float, nsplit: int = 0, prescaled: bool = False,
        fp32_mode: Optional[int] = None, sbuf: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (out (B, R, H*D) in rows.dtype, lse (B, H, R) fp32 natural log).

    ``nsplit``: column splits (0 = auto: split only when R is too small to fill the GPU).
    ``prescaled``: ``rows`` is :func:`prescale` output.  ``fp32_mode``: :func:`fp32_code`
    (None: from ``XDOT_FP32_MODE``).  ``sbuf``: fp32 (exact or split) only, a :func:`score_buffer` the
    raw scores are stored into for :func:`bwd_cols` / :func:`bwd_rows`."""
    bits, flags = _mask_args(mk)
    fm = fp32_code(rows.dtype) if fp32_mode is None else int(fp32_mode)
    return _ext.ops().flash_fwd(rows.contiguous(), _kv(kc), _kv(vc), bits, flags, int(H), float(scale), int(nsplit),
                                bool(prescaled), fm, sbuf)


def bwd_delta(dout: torch.Tensor, out: torch.Tensor, H: int) -> torch.Tensor:
    """δ = rowsum(dO ⊙ O) per (b, h, row): fp32 (B, H, R)."""
    return _ext.ops().flash_bwd_delta(dout.contiguous(), out.contiguous(), int(H))


def bwd_prep(dout: torch.Tensor, out: torch.Tensor, lse: torch.Tensor, H: int):
    """(δ, lse2): δ = rowsum(dO ⊙ O) and the log2-domain LSE, fp32 (B, H, R), in one launch."""
    return _ext.ops().flash_bwd_prep(dout.contiguous(), out.contiguous(), lse.contiguous(), int(H))


def bwd_cols(dout, rows, kc, vc, out, lse, mk: Optional[PackedMask], H: int, scale: float,
             delta: Optional[torch.Tensor] = None, fp32_out: bool = True, prescaled: bool = False,
             lse2: Optional[torch.Tensor] = None, fp32_mode: Optional[int] = None,
             sbuf: Optional[torch.Tensor] = None, dsbuf: Optional[torch.Tensor] = None, passes: int = 3,
             out_dkv: Optional[torch.Tensor] = None):
    """Gathered-side grads -> (packed [d_kc | d_vc] (B, T, 2*H*D), delta (B, H, R)).

    ``delta`` (from :func:`bwd_delta`) is computed here when not given; with ``lse2`` too (both
    from :func:`bwd_prep`) no prep pass is launched here.  The grads are fp32
    (``fp32_out``) or rounded once to the input dtype in the kernel epilogue.  ``sbuf``: the
    forward's :func:`score_buffer`; S is read from it and, without ``dsbuf``, it is OVERWRITTEN
    with dS for :func:`bwd_rows` (run once per forward).  ``dsbuf`` (:func:`score_buffers`): dS
    goes there instead; then ``passes`` may run one pass per call (2 = dQ, which writes dS; 1 = dV)
    with ``out_dkv`` = the first call's output, completed in place."""
    bits, flags = (mk.bits_t, mk.flags) if mk is not None else (None, None)
    return _ext.ops().flash_bwd_cols(dout.contiguous(), rows.contiguous(), _kv(kc), _kv(vc),
                                     out.contiguous(), lse.contiguous(), bits, flags, int(H), float(scale), delta,
                                     bool(fp32_out), bool(prescaled), lse2,
                                     fp32_code(rows.dtype) if fp32_mode is None else int(fp32_mode), sbuf, dsbuf,
                                     int(passes), out_dkv)


def bwd_rows(dout, rows, kc, vc, lse, delta, mk: Optional[PackedMask], H: int, scale: float, nsplit: int = 0,
             prescaled: bool = False, fp32_mode: Optional[int] = None, sbuf: Optional[torch.Tensor] = None,
             dsbuf: Optional[torch.Tensor] = None):
    """Row-side grad (B, R, H*D) in rows.dtype.  ``nsplit`` 0: the launcher's occupancy model
    (column splits so the row kernel fills the GPU; 1 measured 7 % / 32 % slower at N = 1 / 8).
    ``sbuf``: the score buffer after :func:`bwd_cols` wrote dS into it (dK is then its only product);
    with ``dsbuf`` dS is read from there."""
    bits, flags = _mask_args(mk)
    return _ext.ops().flash_bwd_rows(dout.contiguous(), rows.contiguous(), _kv(kc), _kv(vc),
                                     lse.contiguous(), delta.contiguous(), bits, flags, int(H), float(scale),
                                     int(nsplit), bool(prescaled),
                                     fp32_code(rows.dtype) if fp32_mode is None else int(fp32_mode), sbuf, dsbuf)


def bwd(dout: torch.Tensor, rows: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, out: torch.Tensor,
        lse: torch.Tensor, mk: Optional[PackedMask], H: int, scale: float, prescaled: bool = False,
        fp32_mode: Optional[int] = None, sbuf: Optional[torch.Tensor] = None):
    """-> (d_rows (B, R, H*D) rows.dtype, d_kc, d_vc (B, T, H*D) fp32 partial grads).

    ``prescaled``: ``rows`` is :func:`prescale` output (the buffer the forward read); d_rows is
    still the gradient of the unscaled rows.  ``sbuf``: the forward's score buffer (consumed)."""
    dkv, delta = bwd_cols(dout, rows, kc, vc, out, lse, mk, H, scale, prescaled=prescaled, fp32_mode=fp32_mode,
                          sbuf=sbuf)
    drows = bwd_rows(dout, rows, kc, vc, lse, delta, mk, H, scale, prescaled=prescaled, fp32_mode=fp32_mode,
                     sbuf=sbuf)
    C = rows.shape[-1]
    return drows, dkv[..., :C], dkv[..., C:]
