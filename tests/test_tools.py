"""Entry points and tooling on the CPU: ``bench.py`` (the driver's JSON-line contract),
``benchmarks/bench_ops.py`` (reference ``benchmark.py`` CLI + 8-key records, run over gloo
with 2 ranks — BASELINE.json config 1), ``example.py`` (reference ``example.py:1-33``) and
the ``distributed_dot_product`` import shim (reference import lines unchanged)."""
import json
import os
import subprocess
import sys

import pytest

from _dist import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the 8 record keys of the reference's benchmark.py:241-253
REF_KEYS = ("input_memory", "total_time", "peak_memory", "output_memory", "distributed_input_memory",
            "distributed_time", "distributed_peak_memory", "distributed_output_memory")


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "2"
    env["HIP_VISIBLE_DEVICES"] = ""      # CPU path even on a GPU box
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def _run(args, timeout=240):
    p = subprocess.run([sys.executable] + args, cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, f"exit {p.returncode}\nstdout:\n{p.stdout[-3000:]}\nstderr:\n{p.stderr[-3000:]}"
    return p.stdout


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _torchrun(n):
    return ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
            "--master-port", str(free_port())]


def test_bench_contract_cpu():
    out = _run(["bench.py", "--device", "cpu", "--dtype", "fp32", "--seq-len", "128", "--dim", "64",
                "--heads", "4", "--steps", "2", "--warmup", "1"])
    recs = _json_lines(out)
    assert len(recs) == 1, out
    r = recs[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["steps"] == 2 and r["warmup"] == 1
    assert r["value"] > 0 and r["value"] == r["ms_per_step"] and r["higher_is_better"] is False
    assert r["config"]["seq_len"] == 128 and "T=128" in r["metric"]
    assert "synthetic" in r["data"]
    # launch / transport record and the pre-timing numerics check
    assert r["world_size"] == 1 and r["transport"] == "local" and r["rccl_version"] is None
    assert r["gather_chunks"] == 1 and r["local_first"] in (True, False)
    assert 0 <= r["numerics_check_max_rel_err"] < 1e-3  # fp32 on the CPU: the same math


def test_bench_rejects_wrong_world_size():
    """--gpus 2 under a 1-rank LAUNCHER exits 2 instead of timing the wrong job."""
    p = subprocess.run([sys.executable] + _torchrun(1) + ["bench.py", "--gpus", "2", "--device", "cpu", "--backend",
                       "gloo", "--seq-len", "64", "--dim", "32", "--heads", "2", "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode != 0 and "rank(s)" in p.stderr, (p.returncode, p.stderr[-2000:])
    assert not _json_lines(p.stdout)


def test_bench_self_launch_two_ranks():
    """``python bench.py --gpus 2`` with no launcher starts the 2-rank job itself (VERDICT r3
    item 2; reference launch: ``horovodrun -np N``, README.md:77): ONE record, world_size 2."""
    out = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--backend", "gloo", "--dtype", "fp32",
                "--seq-len", "128", "--dim", "64", "--heads", "4", "--steps", "2", "--warmup", "1"])
    recs = _json_lines(out)
    assert len(recs) == 1, out
    assert recs[0]["world_size"] == 2 and recs[0]["n_gpus"] == 2 and recs[0]["config"]["parallelism"] == "sp2"


def test_bench_sweep():
    """``--sweep 1,2``: one record per N from fresh processes, then the scaling summary."""
    out = _run(["bench.py", "--sweep", "1,2", "--device", "cpu", "--backend", "gloo", "--dtype", "fp32",
                "--seq-len", "128", "--dim", "64", "--heads", "4", "--steps", "2", "--warmup", "1", "--no-check"])
    recs = _json_lines(out)
    assert len(recs) == 3, out
    assert [r["n_gpus"] for r in recs[:2]] == [1, 2]
    summ = recs[2]
    assert summ["sweep"] == [1, 2] and set(summ["strong_scaling_efficiency"]) == {"1", "2"}
    assert summ["strong_scaling_efficiency"]["1"] == 1.0


@pytest.mark.parametrize("impl", ["auto", "ring"])
def test_bench_two_ranks_gloo(impl):
    """The driver's N>1 launch line, on the CPU over gloo: ONE JSON line, from rank 0."""
    out = _run(_torchrun(2) + ["bench.py", "--gpus", "2", "--device", "cpu", "--backend", "gloo", "--dtype", "fp32",
                               "--seq-len", "128", "--dim", "64", "--heads", "4", "--steps", "2", "--warmup", "1",
                               "--impl", impl])
    recs = _json_lines(out)
    assert len(recs) == 1, out
    assert recs[0]["n_gpus"] == 2 and recs[0]["config"]["parallelism"] == "sp2"
    assert recs[0]["world_size"] == 2 and recs[0]["transport"] == "gloo"
    assert recs[0]["numerics_check_max_rel_err"] < 1e-3
    # the N>1 breakdown: collectives alone + the compute-only step
    r = recs[0]
    errs = {k: v for k, v in r.items() if k.endswith("_error")}
    assert not errs, errs
    for k in ("allgather_qv", "reduce_scatter_dqv", "allreduce_grads"):
        assert r[f"{k}_ms"] > 0 and r[f"{k}_busbw_gbps"] > 0, k
    assert r["compute_only_ms"] > 0
    assert abs(r["exposed_comm_ms"] - (r["ms_per_step"] - r["compute_only_ms"])) < 1e-3


def test_bench_mismatched_collective_knobs_raise():
    """Ranks launched with different XDOT_GATHER_CHUNKS fail at init (both ranks), not hang."""
    env = _env()
    args = [sys.executable, "-c",
            "import os, sys; os.environ['XDOT_GATHER_CHUNKS'] = str(1 + int(os.environ['RANK'])); "
            "sys.argv = ['bench.py', '--gpus', '2', '--device', 'cpu', '--backend', 'gloo', '--seq-len', '64', "
            "'--dim', '32', '--heads', '2', '--steps', '1', '--warmup', '0']; "
            "import runpy; runpy.run_path('bench.py', run_name='__main__')"]
    # torchrun needs a script path: write the launcher next to the repo's scripts
    launcher = os.path.join(ROOT, "build", "knob_mismatch_launcher.py")
    os.makedirs(os.path.dirname(launcher), exist_ok=True)
    with open(launcher, "w") as f:
        f.write(args[2].replace("; ", "\n"))
    p = subprocess.run([sys.executable] + _torchrun(2) + [launcher], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode != 0, p.stdout[-2000:]
    assert "disagree on collective-shaping flags" in p.stderr + p.stdout, (p.stdout[-2000:], p.stderr[-3000:])


@pytest.mark.parametrize("mode", ["nt", "all", "tn"])
def test_bench_ops_records_gloo(tmp_path, mode):
    """BASELINE.json config 1 (nt, gloo world size 2, T=256, d=64, offset=32) and the other two
    reference modes: a JSON list of records with the reference's 8 keys plus the extras."""
    f = tmp_path / f"{mode}.json"
    out = _run(_torchrun(2) + ["benchmarks/bench_ops.py", "--mode", mode, "--T", "256", "--dim", "64", "--offset",
                               "32", "--iters", "2", "--warmup", "1", "--file", str(f)])
    assert len(_json_lines(out)) == 1
    data = json.loads(f.read_text())
    assert isinstance(data, list) and len(data) == 1
    rec = data[0]
    for k in REF_KEYS:
        assert k in rec, k
    assert rec["world_size"] == 2 and rec["T"] == 256 and rec["D"] == 64 and rec["offset"] == 32
    # fp32 records say which fp32 family ran (exact by default: the reference's precision)
    assert rec["dtype"] != "fp32" or rec["fp32_mode"] == "exact"
    assert rec["ms_p50"] > 0 and rec["distributed_time"] > 0


def test_bench_ops_trial_records(tmp_path):
    """--trials K: the summary record, then K-1 one-call trial records (the reference's files
    hold 100 trials), each with the reference's timing keys."""
    f = tmp_path / "nt.json"
    _run(["benchmarks/bench_ops.py", "--mode", "nt", "--T", "96", "--dim", "16", "--emulate", "3",
          "--iters", "2", "--warmup", "0", "--trials", "4", "--file", str(f)])
    data = json.loads(f.read_text())
    assert len(data) == 4 and "cold_unsynced_s" in data[0]
    assert [r["trial"] for r in data[1:]] == [1, 2, 3]
    for r in data[1:]:
        assert r["distributed_time"] > 0 and r["total_time"] > 0 and r["world_size"] == 3


def test_bench_ops_fwd_bwd_mode_emulated():
    out = _run(["benchmarks/bench_ops.py", "--mode", "leftT_fb", "--T", "96", "--dim", "16", "--emulate", "3",
                "--iters", "1", "--warmup", "0"])
    rec = _json_lines(out)[0]
    assert rec["world_size"] == 3 and rec["emulated"] is True and rec["mode"] == "leftT_fb"


def test_example_runs():
    out = _run(["example.py"], timeout=300)
    assert "rank 0/1" in out and "loss" in out


def test_reference_import_lines():
    """Reference import paths (example.py:10, tests/test_multiplication.py, tests/test_gradient.py)."""
    code = "\n".join([
        "from distributed_dot_product.module import DistributedDotProductAttn",
        "from distributed_dot_product.multiplication.functions import (distributed_matmul_nt,",
        "    distributed_matmul_tn, distributed_matmul_all, distributed_matmul_block)",
        "from distributed_dot_product.multiplication.ops import (RightTransposeMultiplication,",
        "    FullMultiplication, LeftTransposeMultiplication)",
        "from distributed_dot_product.utils.comm import get_world_size, get_rank, is_main_process, synchronize",
        "import distributed_dot_product as d",
        "m = DistributedDotProductAttn(32, num_heads=4)",
        "assert {k.split('.')[0] for k in m.state_dict()} == {'keys', 'queries', 'values', 'composition'}",
        "assert get_world_size() == 1 and get_rank() == 0 and is_main_process()",
        "print('ok', d.__version__)",
    ])
    out = _run(["-c", code])
    assert out.startswith("ok")


def test_packaging_metadata():
    """setup.py reads the version from xdot.VERSION_INFO without importing the package and
    ships the native library as package data (``pip install . --no-build-isolation``)."""
    import os
    import subprocess
    import sys

    import xdot

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "setup.py", "--version"], cwd=root, capture_output=True, text=True,
                       env=dict(os.environ, XDOT_SKIP_NATIVE="1"), timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == xdot.__version__
    src = open(os.path.join(root, "setup.py")).read()
    assert '"_C.so"' in src and "build_py" in src
    assert os.path.exists(os.path.join(root, "pyproject.toml"))


def test_extension_schema_loads_on_cpu():
    """The built xdot/_C.so registers its op schemas at load time (no GPU needed): a schema
    error aborts the process, so load it in a subprocess and expect a clean exit."""
    so = os.path.join(ROOT, "xdot", "_C.so")
    if not os.path.exists(so):
        pytest.skip("xdot/_C.so not built")
    p = subprocess.run([sys.executable, "-c", f"import torch; torch.ops.load_library({so!r}); "
                        "print(len([n for n in dir(torch.ops.xdot) if not n.startswith('_')]))"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]


def test_fp32_mode_codes():
    """XDOT_FP32_MODE -> kernel family code of fp32 operands (16-bit dtypes always 0)."""
    import torch

    from xdot.ops import flash
    from xdot.utils.env import FLAGS

    assert flash.fp32_code(torch.float32, "split") == 1
    assert flash.fp32_code(torch.float32, "exact") == 0
    assert flash.fp32_code(torch.bfloat16, "split") == 0
    old = FLAGS.fp32_mode
    try:
        FLAGS.fp32_mode = "exact"
        assert flash.fp32_code(torch.float32) == 0
        FLAGS.fp32_mode = "bogus"
        with pytest.raises(ValueError):
            flash.fp32_code(torch.float32)
    finally:
        FLAGS.fp32_mode = old


def test_build_id_detects_edited_sources(tmp_path):
    """The extension carries the content hash of csrc/ (xdot/build.py); editing any source makes
    the loader refuse the old binary (a stale _C.so once crashed a GPU run with a
    changed op schema)."""
    import shutil

    import pytest

    from xdot import _ext
    from xdot import build as b

    src = tmp_path / "csrc"
    shutil.copytree(b.CSRC, src)
    h0 = b.tree_hash(str(src))
    assert h0 == b.tree_hash(b.CSRC)
    lib = tmp_path / "_C.so"
    lib.write_bytes(b"\x7fELF..." + b.ID_TAG + h0.encode() + b"\0rest")
    assert b.embedded_id(str(lib)) == h0
    _ext._check_provenance(str(lib), str(src), rebuild=False)  # matching: no error
    f = src / "flash_f32.hip"
    f.write_text(f.read_text() + "\n// edited\n")
    assert b.tree_hash(str(src)) != h0
    with pytest.raises(RuntimeError, match="stale"):
        _ext._check_provenance(str(lib), str(src), rebuild=False)
    # flags are part of the id too
    assert b.tree_hash(b.CSRC, extra=["-O2"]) != b.tree_hash(b.CSRC)
    # the in-tree binary, when built, matches the in-tree sources
    if os.path.exists(b.OUT):
        assert b.embedded_id(b.OUT) == b.tree_hash(b.CSRC)
