"""Shim for reference ``multiplication/ops.py``."""
from xdot.parallel.autograd import (FullMultiplication, LeftTransposeMultiplication,  # noqa: F401
                                    RightTransposeMultiplication)
