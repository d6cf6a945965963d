"""Shim for reference ``multiplication/functions.py`` (same names, ``offset=32`` defaults)."""
from xdot.parallel import functional as _f
from xdot.utils.env import FLAGS
from xdot.utils.profiling import measure  # noqa: F401

DEBUG = FLAGS.debug


def distributed_matmul_nt(left, right, offset=32, **kw):
    return _f.distributed_matmul_nt(left, right, offset, **kw)


def distributed_matmul_all(left, right, offset=32, **kw):
    return _f.distributed_matmul_all(left, right, offset, **kw)


def distributed_matmul_tn(left, right, **kw):
    return _f.distributed_matmul_tn(left, right, **kw)


def distributed_matmul_block(left, right, transpose=False, **kw):
    return _f.distributed_matmul_block(left, right, transpose, **kw)
