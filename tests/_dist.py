"""Multi-process (gloo) and in-process (ThreadComm) harnesses for distributed tests.

``run_gloo(fn, world_size, *args)`` spawns ``world_size`` processes that rendezvous on
127.0.0.1 over gloo, run ``fn(rank, world_size, *args)`` with xdot's default communicator
initialised, and re-raise the first failure in the parent.  ``fn`` must be a top-level
function of an importable module (spawn pickles it by name).
"""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world_size, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world_size), LOCAL_RANK=str(rank))
    try:
        import torch

        torch.set_num_threads(1)
        import xdot.utils.comm as C

        C.init("gloo")
        fn(rank, world_size, *args)
        C.get_comm().barrier()
        C.destroy()
        q.put((rank, None))
    except BaseException:  # noqa: BLE001
        q.put((rank, traceback.format_exc()))
        raise


def run_gloo(fn, world_size, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world_size, port, fn, args, q), daemon=True)
             for r in range(world_size)]
    for p in procs:
        p.start()
    errors = []
    try:
        for _ in range(world_size):
            rank, err = q.get(timeout=timeout)
            if err:
                errors.append(f"rank {rank}:\n{err}")
                break
    finally:
        for p in procs:
            p.join(timeout=5 if errors else 30)
            if p.is_alive():
                p.kill()
    if errors:
        raise AssertionError("\n".join(errors))
