"""Import-compatibility shim: reference import lines keep working on top of :mod:`xdot`.

``from distributed_dot_product.module import DistributedDotProductAttn`` etc. resolve to the
MI355X-native implementations.  Unlike the reference (``module.py:19``, ``utils/comm.py:6``)
importing this package has no side effects: no MPI_Init, no Horovod init.
"""
from xdot import VERSION_INFO, __version__  # noqa: F401
