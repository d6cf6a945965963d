"""Cross-rank consistency checks (race / divergence detection).

The reference relies on every rank issuing the same sequence of named Horovod collectives
and hangs (or silently mixes tensors) when they differ (README "may need one or more runs",
SURVEY §5.2).  With ``XDOT_CHECK=1`` every distributed op first all-gathers a small
fingerprint — op name, call counter, shapes, dtypes, chunk plan — and raises a descriptive
error on the first divergence instead of deadlocking inside RCCL.
"""
from __future__ import annotations

import itertools

import torch

from .env import FLAGS

_counter = itertools.count()


class RankDivergenceError(RuntimeError):
    pass


def fingerprint(op: str, *items) -> tuple:
    fp = [op]
    for it in items:
        if isinstance(it, torch.Tensor):
            fp.append((tuple(it.shape), str(it.dtype)))
        else:
            fp.append(it)
    return tuple(fp)


def check_consistent(comm, op: str, *items, force: bool = False) -> None:
    if not (FLAGS.check or force) or comm.world_size == 1:
        return
    fp = (next(_counter),) + fingerprint(op, *items)
    allfp = comm.all_gather_object(fp)
    if any(f[1:] != allfp[0][1:] for f in allfp):
        lines = "\n".join(f"  rank {r}: {f}" for r, f in enumerate(allfp))
        raise RankDivergenceError(f"xdot: ranks diverged at op {op!r}:\n{lines}")
