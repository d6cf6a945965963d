"""In-tree native build for the gfx950 extension ``xdot/_C.so``.

There is no hipify step and no JIT cache: ``hipcc --offload-arch=gfx950`` compiles every
``csrc/*.hip`` kernel translation unit (no torch headers, seconds each) plus the torch
binding ``csrc/bindings.cpp`` and links them into one shared object that lives next to this
file, so it travels with the repository snapshot to the GPU box.

Usage::

    python -m xdot.build            # incremental
    python -m xdot.build --force    # rebuild everything

The object files are cached under ``build/`` keyed by source + header modification time.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "xdot")
OUT = os.path.join(ROOT, "xdot", "_C.so")
ARCH = "gfx950"  # MI355X only
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch

    base = os.path.dirname(torch.__file__)
    inc = [os.path.join(base, "include"), os.path.join(base, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(base, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h"))


def _stale(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(force: bool = False, verbose: bool = False, jobs: int = 4) -> str:
    """Compile and link ``xdot/_C.so``; returns its path."""
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    # -fno-slp-vectorize: no v_pk_mul/add_f32 beside the MFMAs (packed f32 VALU costs ~13
    # issue cycles per instruction in an MFMA gap vs 4 for each scalar v_fma/v_mul: the
    # softmax / softmax-grad epilogues of the flash kernels are VALU-issue bound)
    from .utils.env import FLAGS

    extra = (FLAGS.hipcc_flags or "-fno-slp-vectorize").split()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", CSRC] + extra + [
              "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-Wno-unused-result", "-Wno-unused-variable"]
    hdrs = _headers()
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs_list.append([HIPCC] + common + ["-c", src, "-o", obj])
    bind = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.o")
    objs.append(bobj)
    if force or _stale(bobj, [bind] + hdrs):
        tinc = []
        for d in inc:
            tinc += ["-isystem", d]
        py_inc = sysconfig.get_paths()["include"]
        jobs_list.append([HIPCC] + common + tinc + ["-isystem", py_inc, "-x", "hip", "-c", bind, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if force or jobs_list or _stale(OUT, objs):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs + [
            "-L", lib, "-Wl,-rpath," + lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-lamdhip64", "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrocprofiler-sdk-roctx"]
        _run(link, verbose)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=4)
    a = ap.parse_args(argv)
    path = build(force=a.force, verbose=a.verbose, jobs=a.jobs)
    print(path)


if __name__ == "__main__":
    sys.exit(main())
