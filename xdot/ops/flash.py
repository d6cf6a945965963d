"""Python face of the flash-attention kernels (``csrc/flash_fwd.hip``, ``csrc/flash_bwd.hip``,
``csrc/mask_pack.hip``).

Tensors are head-interleaved: ``rows`` (B, R, H*D) local query-side rows, ``kc``/``vc``
(N, B, Rc, H*D) the rank-major gathered key/value side (T = N*Rc columns).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import _ext


class PackedMask:
    """Boolean (B, R, T) mask compressed to per-row bit words + per-tile flags."""

    __slots__ = ("bits", "flags", "shape")

    def __init__(self, bits: torch.Tensor, flags: torch.Tensor, shape):
        self.bits, self.flags, self.shape = bits, flags, tuple(shape)

    @property
    def nothing_masked(self) -> bool:  # host sync; diagnostics only
        return bool((self.flags == 0).all())


def prepare_mask(mask: Optional[torch.Tensor], B: int, R: int, T: int) -> Optional[PackedMask]:
    if mask is None:
        return None
    if tuple(mask.shape) != (B, R, T):
        raise ValueError(f"mask must be (B, R, T) = {(B, R, T)}, got {tuple(mask.shape)}")
    bits, flags = _ext.ops().mask_pack(mask.to(torch.bool).contiguous())
    return PackedMask(bits, flags, mask.shape)


def _mask_args(mk: Optional[PackedMask]):
    return (mk.bits, mk.flags) if mk is not None else (None, None)


def fwd(rows: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, mk: Optional[PackedMask], H: int,
        scale: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (out (B, R, H*D) in rows.dtype, lse (B, H, R) fp32 natural log)."""
    bits, flags = _mask_args(mk)
    return _ext.ops().flash_fwd(rows.contiguous(), kc.contiguous(), vc.contiguous(), bits, flags, int(H), float(scale))


def bwd(dout: torch.Tensor, rows: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, out: torch.Tensor,
        lse: torch.Tensor, mk: Optional[PackedMask], H: int, scale: float):
    """-> (d_rows (B, R, H*D) rows.dtype, d_kc, d_vc (N, B, Rc, H*D) fp32 partials)."""
    bits, flags = _mask_args(mk)
    return _ext.ops().flash_bwd(dout.contiguous(), rows.contiguous(), kc.contiguous(), vc.contiguous(),
                                out.contiguous(), lse.contiguous(), bits, flags, int(H), float(scale))
