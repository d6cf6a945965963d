"""Loader for the in-tree gfx950 extension ``xdot/_C.so`` (``torch.ops.xdot.*``).

Policy: GPU tensors run on the HIP kernels.  If the extension is missing on a machine with
a GPU, xdot raises (set ``XDOT_ALLOW_TORCH_FALLBACK=1`` to permit the slow torch path, e.g.
for debugging); CPU tensors always use the torch reference implementations.
"""
from __future__ import annotations

import os
import threading

import torch

from .utils.env import FLAGS

# XDOT_EXT_PATH: load a differently built copy (A/B kernel experiments in one GPU session)
_LIB = FLAGS.ext_path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C.so")
_lock = threading.Lock()
_state = {"loaded": False, "error": None}


def lib_path() -> str:
    return _LIB


def provenance(lib: str = None, csrc: str = None):
    """(build id embedded in ``lib``, hash of the ``csrc`` tree): equal when the binary was built
    from exactly these sources and flags (:func:`xdot.build.tree_hash`)."""
    from . import build as _b

    return _b.embedded_id(lib or _LIB), _b.tree_hash(csrc or _b.CSRC)


def _check_provenance(lib: str = None, csrc: str = None, rebuild: bool = None) -> None:
    """Refuse (or rebuild) an in-tree ``_C.so`` that was not built from the sources next to it:
    a stale binary either crashes on a changed op schema or silently runs old kernels.  Skipped
    for ``XDOT_EXT_PATH`` builds (A/B experiments) and when the sources are not present."""
    from . import build as _b

    csrc = csrc or _b.CSRC
    if (FLAGS.ext_path and lib is None) or not os.path.isdir(csrc):
        return
    have, want = provenance(lib, csrc)
    if have == want:
        return
    rebuild = FLAGS.auto_rebuild if rebuild is None else rebuild
    if rebuild and lib is None and os.path.exists(_b.HIPCC):
        import sys

        print(f"xdot: {_LIB} build id {have} != sources {want}: rebuilding", file=sys.stderr, flush=True)
        _b.build()
        have = _b.embedded_id(_LIB)
        if have == want:
            return
    raise RuntimeError(f"xdot: {lib or _LIB} is stale (build id {have}, csrc/ tree {want}); rebuild it with "
                       "`python -m xdot.build` (or set XDOT_EXT_PATH to load a specific build)")


def load(build_if_missing: bool = False) -> bool:
    """Load ``_C.so`` once (after :func:`_check_provenance`).  Returns True on success."""
    if _state["loaded"]:
        return True
    with _lock:
        if _state["loaded"]:
            return True
        if not os.path.exists(_LIB) and build_if_missing:
            from . import build as _b

            _b.build()
        if not os.path.exists(_LIB):
            _state["error"] = f"{_LIB} not built (run `python -m xdot.build`)"
            return False
        _check_provenance()
        try:
            torch.ops.load_library(_LIB)
            _state["loaded"] = True
        except Exception as e:  # noqa: BLE001
            _state["error"] = f"failed to load {_LIB}: {e}"
            return False
    return True


def available() -> bool:
    return load()


_tls = threading.local()
BACKENDS = ("auto", "hip", "torch")


def current_backend() -> str:
    """Compute backend in effect on this thread: a :func:`backend` override, else
    ``XDOT_BACKEND`` (``auto`` | ``hip`` | ``torch``)."""
    return getattr(_tls, "backend", None) or FLAGS.backend


class backend:
    """``with _ext.backend('torch'):`` — override the compute backend on this thread (what the
    ``backend=`` argument of :class:`xdot.DistributedDotProductAttn` does).  ``None`` / ``'auto'``
    keep the process default.  Autograd runs backward on its own thread, so the custom
    Functions record the backend in forward and re-enter it in backward (:func:`pinned`)."""

    def __init__(self, b: str = None):
        if b is not None and b not in BACKENDS:
            raise ValueError(f"backend must be one of {BACKENDS}, got {b!r}")
        self.b = None if b in (None, "auto") else b

    def __enter__(self):
        self.prev = getattr(_tls, "backend", None)
        if self.b is not None:
            _tls.backend = self.b
        return self

    def __exit__(self, *exc):
        _tls.backend = self.prev
        return False


def pinned(fn):
    """Decorator for ``forward(ctx, ...)`` / ``backward(ctx, ...)`` of a custom autograd Function:
    forward records :func:`current_backend`, backward runs under it."""
    import functools

    @functools.wraps(fn)
    def wrap(ctx, *args):
        if fn.__name__ == "forward":
            ctx.xdot_backend = getattr(_tls, "backend", None)
            return fn(ctx, *args)
        with backend(getattr(ctx, "xdot_backend", None)):
            return fn(ctx, *args)

    return wrap


def use_hip(*tensors: torch.Tensor) -> bool:
    """Decide whether GPU tensors go to the HIP kernels.  Raises if they should but the
    extension is not loadable (no silent fallback on a GPU box)."""
    if not any(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors):
        return False
    if current_backend() == "torch":
        return False
    if load():
        return True
    if FLAGS.allow_torch_fallback:
        return False
    raise RuntimeError(f"xdot: HIP extension unavailable for GPU tensors: {_state['error']}")


def ops():
    if not load():
        raise RuntimeError(f"xdot: HIP extension unavailable: {_state['error']}")
    return torch.ops.xdot
