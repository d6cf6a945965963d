"""Model families built on the distributed products."""
from .attention import DistributedDotProductAttn  # noqa: F401
