"""Build the gfx950 kernel library in-tree: ``distributed_training_compare_jax_amd/_dtc_kernels.so``.

    python -m distributed_training_compare_jax_amd.csrc.build [--force] [-j N] [--debug]

Each ``csrc/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` (cross-compiles without a
GPU) and the objects are linked into one shared library with a C ABI (``ops/_native.py``).
The host-only runtime sources (``csrc/*.cpp``: the native data pipeline) are compiled by the host
C++ compiler into ``_dtc_host.so`` (no GPU code, loadable on CPU-only machines).
Rebuilds only when a source/header hash changed; :data:`STATUS` records whether the last
:func:`build` compiled or reused the library (``__graft_entry__.build()`` prints it).

Debug variant (``--debug`` or ``DTC_DEBUG=1``): ``-O1 -g -DDTC_DEBUG`` into ``_dtc_kernels_debug.so``
(selected at run time with ``DTC_KERNEL_LIB=<that path>``): ``DTC_ASSERT`` bounds checks in the
kernels (``common.h``) become device asserts, and the host entry points validate shapes/alignment.
"""

from __future__ import annotations

import argparse
import glob
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
OUT = os.path.join(PKG, "_dtc_kernels.so")
HOST_OUT = os.path.join(PKG, "_dtc_host.so")
BUILD = os.path.join(HERE, "build")
ARCH = os.environ.get("DTC_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-Wno-unused-result"]
DEBUG_FLAGS = ["-O1", "-g", "-DDTC_DEBUG", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
               "-Wno-unused-result"]
DEBUG_OUT = os.path.join(PKG, "_dtc_kernels_debug.so")
FILE_FLAGS = {}  # per-file extra hipcc options (basename -> list)
STATUS = {"kernels": None, "host": None}  # "compiled" | "reused" after build()


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm not installed?)")


def _digest(paths, flags=FLAGS) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(os.path.basename(p).encode())  # path-independent: the box copy reuses this build
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def build_host(force: bool = False, verbose: bool = False) -> str:
    """csrc/*.cpp -> _dtc_host.so (host C++ only)."""
    srcs = sorted(glob.glob(os.path.join(HERE, "*.cpp")))
    os.makedirs(BUILD, exist_ok=True)
    stamp = os.path.join(BUILD, "stamp_host")
    dig = _digest(srcs)
    if not force and os.path.exists(HOST_OUT) and os.path.exists(stamp) and open(stamp).read() == dig:
        STATUS["host"] = "reused"
        return HOST_OUT
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++") or "/opt/rocm/llvm/bin/clang++"
    tmp = HOST_OUT + ".tmp"
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-o", tmp, *srcs]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host build failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, HOST_OUT)
    with open(stamp, "w") as f:
        f.write(dig)
    STATUS["host"] = "compiled"
    return HOST_OUT


def build(force: bool = False, jobs: int = 8, verbose: bool = False, debug: bool = None) -> str:
    if debug is None:
        debug = os.environ.get("DTC_DEBUG", "0") == "1"
    build_host(force, verbose)
    srcs = sorted(glob.glob(os.path.join(HERE, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(HERE, "*.h")))
    flags, out, tag = (DEBUG_FLAGS, DEBUG_OUT, "_debug") if debug else (FLAGS, OUT, "")
    bdir = os.path.join(BUILD, "debug") if debug else BUILD
    os.makedirs(bdir, exist_ok=True)
    stamp = os.path.join(bdir, "stamp" + tag)
    dig = _digest(srcs + hdrs, flags + [f"{k}:{' '.join(v)}" for k, v in sorted(FILE_FLAGS.items())])
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == dig:
        STATUS["kernels"] = "reused"
        return out
    cc = hipcc()

    def comp(src):
        obj = os.path.join(bdir, os.path.basename(src).replace(".hip", ".o"))
        cmd = [cc, *flags, *FILE_FLAGS.get(os.path.basename(src), []), "-I", HERE, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-6000:]}")
        return obj

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(comp, srcs))
    tmp = out + ".tmp"
    r = subprocess.run([cc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", tmp, *objs], capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(dig)
    STATUS["kernels"] = "compiled"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true", help="-O1 -g -DDTC_DEBUG variant (_dtc_kernels_debug.so)")
    a = ap.parse_args()
    out = build(a.force, a.jobs, a.verbose, debug=a.debug or None)
    print(f"{out} ({STATUS['kernels']}; host library {STATUS['host']})")


if __name__ == "__main__":
    sys.exit(main())
