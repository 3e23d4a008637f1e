"""Build the gfx950 kernel library in-tree: ``distributed_training_compare_jax_amd/_dtc_kernels.so``.

    python -m distributed_training_compare_jax_amd.csrc.build [--force] [-j N]

Each ``csrc/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` (cross-compiles without a
GPU) and the objects are linked into one shared library with a C ABI (``ops/_native.py``).
The host-only runtime sources (``csrc/*.cpp``: the native data pipeline) are compiled by the host
C++ compiler into ``_dtc_host.so`` (no GPU code, loadable on CPU-only machines).
Rebuilds only when a source/header hash changed.
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


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm not installed?)")


def _digest(paths) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(p.encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()


def build_host(force: bool = False, verbose: bool = False) -> str:
    """csrc/*.cpp -> _dtc_host.so (host C++ only)."""
    srcs = sorted(glob.glob(os.path.join(HERE, "*.cpp")))
    os.makedirs(BUILD, exist_ok=True)
    stamp = os.path.join(BUILD, "stamp_host")
    dig = _digest(srcs)
    if not force and os.path.exists(HOST_OUT) and os.path.exists(stamp) and open(stamp).read() == dig:
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
    return HOST_OUT


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    build_host(force, verbose)
    srcs = sorted(glob.glob(os.path.join(HERE, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(HERE, "*.h")))
    os.makedirs(BUILD, exist_ok=True)
    stamp = os.path.join(BUILD, "stamp")
    dig = _digest(srcs + hdrs)
    if not force and os.path.exists(OUT) and os.path.exists(stamp) and open(stamp).read() == dig:
        return OUT
    cc = hipcc()

    def comp(src):
        obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
        cmd = [cc, *FLAGS, "-I", HERE, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-6000:]}")
        return obj

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(comp, srcs))
    tmp = OUT + ".tmp"
    r = subprocess.run([cc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", tmp, *objs], capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, OUT)
    with open(stamp, "w") as f:
        f.write(dig)
    return OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    out = build(a.force, a.jobs, a.verbose)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
