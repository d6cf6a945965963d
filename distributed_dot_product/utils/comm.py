"""Shim for reference ``utils/comm.py`` (torch.distributed instead of Horovod/MPI)."""
from xdot.utils.comm import get_rank, get_world_size, is_main_process, synchronize  # noqa: F401
