"""RCCL-only code paths of ``TorchDistComm`` (in-place all-gather, grouped all-gathers and
all-reduces through ``dist._coalescing_manager``, native average, GradSync's in-place bucket
reduce) on device memory under torchrun: ``scripts/rccl_api_check.py`` with one rank on the GPU
box (gloo, which the CPU suite uses, never reaches these paths)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun_one(script):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "scripts", script)]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    return p.stdout


def test_rccl_paths_world_one():
    assert "rccl-api-ok 1" in _torchrun_one("rccl_api_check.py")


def test_rccl_collectives_under_graph_capture():
    """all-reduce / all-gather / reduce-scatter of TorchDistComm captured in one HIP graph and
    replayed with new inputs (GraphedStep's contract for a real communicator)."""
    assert "rccl-graph-ok 1" in _torchrun_one("rccl_graph_check.py")
