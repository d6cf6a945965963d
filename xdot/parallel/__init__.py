"""Sequence-parallel distributed products, their autograd ops, fused seq-parallel attention,
chunk schedules and replicated-parameter (SP gradient) helpers."""
from .functional import (distributed_matmul_nt, distributed_matmul_all, distributed_matmul_tn,  # noqa: F401
                         distributed_matmul_block, gather_sequence)
from .autograd import RightTransposeMultiplication, FullMultiplication, LeftTransposeMultiplication  # noqa: F401
from .attention import seq_parallel_attention, SeqParallelAttention  # noqa: F401
from .data_parallel import broadcast_parameters, allreduce_gradients, GradSync  # noqa: F401
from .schedule import plan_chunks, auto_offset  # noqa: F401
