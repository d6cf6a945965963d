"""Autograd wrappers of the distributed products (reference: ``multiplication/ops.py:19-71``).

Each ``.apply(left, right, offset)`` returns the local row block and backpropagates with the
other two distributed products, exactly like the reference — with three fixes:

* ``offset`` is forwarded in the forward pass too (reference ``ops.py:25,45`` drops it);
* ``LeftTransposeMultiplication`` returns the *correct* left gradient ``nt(right, dC)``; the
  reference returns ``nt(dC, right)`` = the transposed block (``ops.py:69``).
  ``compat_reference_bug=True`` reproduces the old value for bit-compatibility studies;
* outputs keep the input dtype (bf16/fp16 work; the reference crashes in bf16).

The communicator active at forward time is captured and reused in backward (autograd runs
backward on its own thread, where a thread-local default would not be visible).
"""
from __future__ import annotations

from typing import Any, Optional

import torch
from torch import Tensor

from .. import _ext
from ..utils import comm as _comm
from .functional import distributed_matmul_all, distributed_matmul_nt, distributed_matmul_tn

__all__ = ["RightTransposeMultiplication", "FullMultiplication", "LeftTransposeMultiplication"]


class RightTransposeMultiplication(torch.autograd.Function):
    """``C = A·Bᵀ`` (local (P,R,D) x (P,R,D) -> (P,R,T)).  Reference ``ops.py:19-37``."""

    @staticmethod
    @_ext.pinned
    def forward(ctx: Any, left: Tensor, right: Tensor, offset: Optional[int] = None,
                comm: Optional[_comm.Communicator] = None) -> Tensor:
        comm = comm or _comm.get_comm()
        ctx.save_for_backward(left, right)
        ctx.offset, ctx.comm = offset, comm
        return distributed_matmul_nt(left, right, offset, comm=comm)

    @staticmethod
    @_ext.pinned
    def backward(ctx: Any, grad: Tensor):
        left, right = ctx.saved_tensors
        gl = gr = None
        if ctx.needs_input_grad[1]:
            gr = distributed_matmul_tn(grad, left, comm=ctx.comm)
        if ctx.needs_input_grad[0]:
            gl = distributed_matmul_all(grad, right, ctx.offset, comm=ctx.comm)
        return gl, gr, None, None


class FullMultiplication(torch.autograd.Function):
    """``C = A·B`` (local (P,R,T) x (P,R,D) -> (P,R,D)).  Reference ``ops.py:40-54``."""

    @staticmethod
    @_ext.pinned
    def forward(ctx: Any, left: Tensor, right: Tensor, offset: Optional[int] = None,
                comm: Optional[_comm.Communicator] = None) -> Tensor:
        comm = comm or _comm.get_comm()
        ctx.save_for_backward(left, right)
        ctx.offset, ctx.comm = offset, comm
        return distributed_matmul_all(left, right, offset, comm=comm)

    @staticmethod
    @_ext.pinned
    def backward(ctx: Any, grad: Tensor):
        left, right = ctx.saved_tensors
        gl = gr = None
        if ctx.needs_input_grad[0]:
            gl = distributed_matmul_nt(grad, right, ctx.offset, comm=ctx.comm)
        if ctx.needs_input_grad[1]:
            gr = distributed_matmul_tn(left, grad, comm=ctx.comm)
        return gl, gr, None, None


class LeftTransposeMultiplication(torch.autograd.Function):
    """``C = Aᵀ·B`` (local (P,R,T) x (P,R,D) -> (P,R,D)).  Reference ``ops.py:57-71``."""

    compat_reference_bug = False

    @staticmethod
    @_ext.pinned
    def forward(ctx: Any, left: Tensor, right: Tensor, offset: Optional[int] = None,
                comm: Optional[_comm.Communicator] = None) -> Tensor:
        comm = comm or _comm.get_comm()
        ctx.save_for_backward(left, right)
        ctx.offset, ctx.comm = offset, comm
        return distributed_matmul_tn(left, right, comm=comm)

    @staticmethod
    @_ext.pinned
    def backward(ctx: Any, grad: Tensor):
        left, right = ctx.saved_tensors
        gl = gr = None
        if ctx.needs_input_grad[0]:
            if LeftTransposeMultiplication.compat_reference_bug:
                gl = distributed_matmul_nt(grad, right, ctx.offset, comm=ctx.comm)
            else:  # dA = B·dCᵀ, local rows: nt(B_local, dC_local)
                gl = distributed_matmul_nt(right, grad, ctx.offset, comm=ctx.comm)
        if ctx.needs_input_grad[1]:
            gr = distributed_matmul_all(left, grad, ctx.offset, comm=ctx.comm)
        return gl, gr, None, None
