"""In-tree native build for the gfx950 extension ``xdot/_C.so``.

There is no hipify step and no JIT cache: ``hipcc --offload-arch=gfx950`` compiles every
``csrc/*.hip`` kernel translation unit (no torch headers, seconds each) plus the torch
binding ``csrc/bindings.cpp`` and links them into one shared object that lives next to this
file, so it travels with the repository snapshot to the GPU box.

Usage::

    python -m xdot.build            # incremental
    python -m xdot.build --force    # rebuild everything

The object files are cached under ``build/``, keyed by a content hash of their source, every
header and the compile flags.  Provenance: the link embeds :func:`tree_hash` (sha256 of every
file in ``csrc/`` plus the flags) as the string ``XDOT_BUILD_ID=<hash>`` in ``_C.so``
(``torch.ops.xdot.build_id()``); :mod:`xdot._ext` compares it with the tree before loading and
rebuilds (or raises) on a mismatch, so a stale binary can never run.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shlex
import shutil
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


def _flags() -> list:
    from .utils.env import FLAGS

    # -fno-slp-vectorize: no v_pk_mul/add_f32 beside the MFMAs (packed f32 VALU costs ~13
    # issue cycles per instruction in an MFMA gap vs 4 for each scalar v_fma/v_mul: the
    # softmax / softmax-grad epilogues of the flash kernels are VALU-issue bound)
    return (FLAGS.hipcc_flags or "-fno-slp-vectorize").split()


def tree_hash(csrc: str = CSRC, extra=None) -> str:
    """sha256 of every file in ``csrc`` (names and contents, sorted) + the target and flags: the
    build id ``_C.so`` must carry to be loaded."""
    h = hashlib.sha256()
    h.update(f"arch={ARCH};flags={' '.join(_flags() if extra is None else extra)}\n".encode())
    for f in sorted(os.listdir(csrc)):
        path = os.path.join(csrc, f)
        if not os.path.isfile(path):
            continue
        h.update(f.encode() + b"\0")
        with open(path, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()


ID_TAG = b"XDOT_BUILD_ID="


def embedded_id(lib: str):
    """The build id compiled into a built extension (read from the file, WITHOUT loading it:
    a loaded library cannot be replaced in-process), or None."""
    try:
        with open(lib, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(ID_TAG)
    if i < 0:
        return None
    v = data[i + len(ID_TAG):i + len(ID_TAG) + 64]
    return v.decode("ascii", "replace")


def _dep_hash(src: str, hdrs, flags) -> str:
    h = hashlib.sha256(" ".join(flags).encode())
    for f in [src] + sorted(hdrs):
        with open(f, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()


def _stale(obj: str, key: str) -> bool:
    """An object is rebuilt unless the content hash of its inputs matches the one it was built from."""
    if not os.path.exists(obj) or not os.path.exists(obj + ".key"):
        return True
    with open(obj + ".key") as fh:
        return fh.read().strip() != key


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
    extra = _flags()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", CSRC] + extra + [
              "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-Wno-unused-result", "-Wno-unused-variable"]
    hdrs = _headers()
    jobs_list = []  # (command, object, key)
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        key = _dep_hash(src, hdrs, common)
        if force or _stale(obj, key):
            jobs_list.append(([HIPCC] + common + ["-c", src, "-o", obj], obj, key))
    bind = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.o")
    objs.append(bobj)
    bkey = _dep_hash(bind, hdrs, common)
    if force or _stale(bobj, bkey):
        tinc = []
        for d in inc:
            tinc += ["-isystem", d]
        py_inc = sysconfig.get_paths()["include"]
        jobs_list.append(([HIPCC] + common + tinc + ["-isystem", py_inc, "-x", "hip", "-c", bind, "-o", bobj],
                          bobj, bkey))
    # the provenance string: a one-line translation unit, so a source edit recompiles only it
    bid = tree_hash()
    idsrc = os.path.join(BUILD, "build_id.cpp")
    idobj = os.path.join(BUILD, "build_id.o")
    objs.append(idobj)
    if force or _stale(idobj, bid):
        with open(idsrc, "w") as fh:
            fh.write("// generated by xdot/build.py: sha256 of csrc/* + flags (xdot._ext checks it on load)\n"
                     f'extern "C" __attribute__((used, visibility("default"))) const char xdot_build_id[] = '
                     f'"{ID_TAG.decode()}{bid}";\n')
        jobs_list.append(([shutil.which("g++") or HIPCC, "-O2", "-fPIC", "-c", idsrc, "-o", idobj], idobj, bid))

    def work(job):
        cmd, obj, key = job
        if os.path.exists(obj + ".key"):
            os.remove(obj + ".key")
        _run(cmd, verbose)
        with open(obj + ".key", "w") as fh:
            fh.write(key)

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(work, jobs_list))
    if force or jobs_list or embedded_id(OUT) != bid:
        tmp = OUT + ".tmp"
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            "-L", lib, "-Wl,-rpath," + lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-lamdhip64", "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrocprofiler-sdk-roctx"]
        _run(link, verbose)
        os.replace(tmp, OUT)  # atomic: a concurrent loader never sees a half-written library
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
