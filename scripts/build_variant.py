"""Build the kernel library with extra compile flags into another path (A/B of compile-time
variants; select it at run time with DTC_KERNEL_LIB=<path>).

    python scripts/build_variant.py variants/_dtc_x.so -DDTC_DEEP_PREFETCH_MAX=4096
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_training_compare_jax_amd.csrc import build as B  # noqa: E402

out, extra = sys.argv[1], sys.argv[2:]
tag = os.path.splitext(os.path.basename(out))[0]
bdir = os.path.join(B.BUILD, "variant_" + tag)
os.makedirs(bdir, exist_ok=True)
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
cc = B.hipcc()


def comp(src):
    obj = os.path.join(bdir, os.path.basename(src).replace(".hip", ".o"))
    r = subprocess.run([cc, *B.FLAGS, *extra, "-I", B.HERE, "-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-4000:])
    return obj


with ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(comp, sorted(glob.glob(os.path.join(B.HERE, "*.hip")))))
subprocess.run([cc, "-shared", f"--offload-arch={B.ARCH}", "-fPIC", "-o", out, *objs], check=True)
print(out)
