"""Device operators: gfx950 HIP kernels behind ``torch.ops.xdot`` + torch reference paths."""
from .gemm import strided_gemm, nt_chunk_into, all_chunk_into, tn_partials_into, matmul  # noqa: F401
from .softmax import (ScaleMaskSoftmax, scale_mask_softmax, scale_mask_softmax_fwd,  # noqa: F401
                      scale_mask_softmax_bwd)
from .linear import linear, weight_grad  # noqa: F401
from .optim import FusedAdamW  # noqa: F401
from .loss import mse_loss, MSELoss  # noqa: F401
