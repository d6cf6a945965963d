"""Timing / memory instrumentation.

:func:`measure` is the sync-correct successor of the reference's debug decorator
(reference: ``distributed_dot_product/multiplication/functions.py:24-41``, gated by
``DISTRIBUTED_DOT_DEBUG``): the reference reads ``time.time()`` around asynchronous GPU work
without a device sync, so it measures launch overhead.  Here the elapsed time comes from HIP
events on the current stream (only when debugging is on, so the hot path pays nothing), and
every op is wrapped in a ``torch.profiler.record_function`` range so rocprofv3 / torch
profiler traces carry op names.
"""
from __future__ import annotations

import functools
import logging
import time
from contextlib import contextmanager

import torch

from .env import FLAGS

log = logging.getLogger("xdot")


def _shape(x):
    return tuple(x.shape) if isinstance(x, torch.Tensor) else type(x).__name__


def measure(fn):
    """Decorator: named profiler range always; shapes/time/HBM delta when ``FLAGS.debug``."""
    name = f"xdot::{fn.__name__}"

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        if not FLAGS.debug:
            with torch.profiler.record_function(name):
                return fn(*args, **kwargs)
        cuda = any(isinstance(a, torch.Tensor) and a.is_cuda for a in args)
        if cuda:
            torch.cuda.synchronize()
            m0 = torch.cuda.max_memory_allocated()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        t0 = time.perf_counter()
        with torch.profiler.record_function(name):
            out = fn(*args, **kwargs)
        msg = f"{fn.__name__} - " + ", ".join(str(_shape(a)) for a in args[:2])
        if cuda:
            e1.record()
            e1.synchronize()
            dm = torch.cuda.max_memory_allocated() - m0
            msg += f" | {e0.elapsed_time(e1):.3f} ms (hip events) | peak HBM delta {dm / 2**20:.1f} MiB"
        else:
            msg += f" | {(time.perf_counter() - t0) * 1e3:.3f} ms"
        log.warning(msg) if log.handlers else print(msg, flush=True)
        return out

    return wrapper


@contextmanager
def cuda_timer(store: dict, key: str, enabled: bool = True):
    """Accumulate the device time of a region (ms) into ``store[key]`` (HIP events)."""
    if not enabled or not torch.cuda.is_available():
        yield
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    yield
    e1.record()
    e1.synchronize()
    store[key] = store.get(key, 0.0) + e0.elapsed_time(e1)
