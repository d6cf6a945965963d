"""xdot — sequence-parallel dot-product attention for AMD Instinct MI355X (gfx950).

A from-scratch MI355X-native library with the capabilities of andfoy/py-distributed-dot-product:
distributed A·Bᵀ / A·B / Aᵀ·B over a time axis sharded into contiguous T/N row blocks, their
autograd ops, and the multi-head ``DistributedDotProductAttn`` module — on PyTorch-ROCm,
hand-written CDNA4 HIP kernels (``xdot/_C.so``) and RCCL over xGMI.
"""
VERSION_INFO = (0, 1, 0)
__version__ = ".".join(map(str, VERSION_INFO))

from .utils.comm import (init, get_rank, get_world_size, is_main_process, synchronize,  # noqa: E402,F401
                         get_comm, use_comm, LocalComm, ThreadGroup)
from .parallel import (distributed_matmul_nt, distributed_matmul_all, distributed_matmul_tn,  # noqa: E402,F401
                       distributed_matmul_block, RightTransposeMultiplication, FullMultiplication,
                       LeftTransposeMultiplication, seq_parallel_attention, broadcast_parameters,
                       allreduce_gradients, GradSync, gather_sequence)
from .models import DistributedDotProductAttn  # noqa: E402,F401
from .ops import scale_mask_softmax, linear, FusedAdamW, MSELoss, mse_loss  # noqa: E402,F401
