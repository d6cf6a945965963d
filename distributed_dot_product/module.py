"""Shim for reference ``distributed_dot_product/module.py``."""
from xdot.models.attention import DistributedDotProductAttn  # noqa: F401

__all__ = ["DistributedDotProductAttn"]
