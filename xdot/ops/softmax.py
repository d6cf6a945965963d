"""Fused scale + mask + softmax (``csrc/softmax.hip``) with its autograd Function.

Reference (``distributed_dot_product/module.py:65-67``)::

    projection = projection / math.sqrt(self.dim)
    projection = projection.masked_fill(attn_mask, -float('inf'))
    attn = torch.softmax(projection, dim=-1)

three full passes (plus three in backward) over a (B, H, T/N, T) block; here one pass each way.
``mask`` is the module's (B, R, T) bool mask broadcast over the H heads of a (B, H, R, T)
score tensor, or any mask whose shape equals the scores' shape.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .. import _ext


def _mask_map(scores: torch.Tensor, mask: torch.Tensor):
    """Return (mask_2d, mdiv, mmul, mmod) mapping score rows to mask rows."""
    T = scores.shape[-1]
    rows = scores.numel() // max(T, 1)
    if mask.shape == scores.shape:
        return mask.contiguous(), rows, 0, rows
    if scores.dim() == 4 and mask.dim() == 3 and mask.shape[0] == scores.shape[0] \
            and mask.shape[1:] == scores.shape[2:]:
        B, H, R, _ = scores.shape
        return mask.contiguous(), H * R, R, R
    if scores.dim() == 4 and mask.dim() == 4 and mask.shape[1] == 1:
        B, H, R, _ = scores.shape
        return mask.reshape(mask.shape[0], R, T).contiguous(), H * R, R, R
    raise ValueError(f"unsupported mask shape {tuple(mask.shape)} for scores {tuple(scores.shape)}")


def _torch_mask(scores, mask):
    if mask.dim() == 3 and scores.dim() == 4:
        mask = mask.unsqueeze(1)
    return mask


def scale_mask_softmax_fwd(scores: torch.Tensor, mask: Optional[torch.Tensor], scale: float) -> torch.Tensor:
    if _ext.use_hip(scores) and scores.dtype in (torch.float32, torch.bfloat16, torch.float16):
        s = scores.contiguous()
        if mask is None:
            return _ext.ops().softmax_fwd(s, None, float(scale), 1, 0, 1)
        m, mdiv, mmul, mmod = _mask_map(s, mask.to(device=s.device, dtype=torch.bool))
        return _ext.ops().softmax_fwd(s, m, float(scale), mdiv, mmul, mmod)
    x = scores * scale if scale != 1.0 else scores
    if mask is not None:
        x = x.masked_fill(_torch_mask(scores, mask), -float("inf"))
    return torch.softmax(x, dim=-1)


def scale_mask_softmax_bwd(y: torch.Tensor, dy: torch.Tensor, scale: float) -> torch.Tensor:
    if _ext.use_hip(y) and y.dtype in (torch.float32, torch.bfloat16, torch.float16):
        return _ext.ops().softmax_bwd(y.contiguous(), dy.contiguous().to(y.dtype), float(scale))
    cdt = torch.float64 if y.dtype == torch.float64 else torch.float32
    yf, dyf = y.to(cdt), dy.to(cdt)
    return (scale * yf * (dyf - (dyf * yf).sum(-1, keepdim=True))).to(y.dtype)


class ScaleMaskSoftmax(torch.autograd.Function):
    """y = softmax(scale * x, masked -> -inf); one fused kernel per direction on GPU."""

    @staticmethod
    @_ext.pinned
    def forward(ctx, scores, mask, scale):
        y = scale_mask_softmax_fwd(scores, mask, scale)
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    @_ext.pinned
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return scale_mask_softmax_bwd(y, dy, ctx.scale), None, None


def scale_mask_softmax(scores: torch.Tensor, mask: Optional[torch.Tensor] = None,
                       scale: Optional[float] = None, head_dim: Optional[int] = None) -> torch.Tensor:
    """Differentiable fused softmax.  ``scale`` defaults to ``1/sqrt(head_dim)`` if given."""
    if scale is None:
        scale = 1.0 / math.sqrt(head_dim) if head_dim else 1.0
    return ScaleMaskSoftmax.apply(scores, mask, float(scale))
