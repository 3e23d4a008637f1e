"""Where the resident attention backward spends its time: per-block wall-clock stamps from a
diagnostic build (scripts/build_variant.py variants/_dtc_stamps.so -DDTC_ATTN_STAMPS).

    DTC_KERNEL_LIB=variants/_dtc_stamps.so python scripts/attn_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import _native as N  # noqa: E402
from distributed_training_compare_jax_amd.ops import attention as A  # noqa: E402

B, T, H, HD = 8, 512, 16, 32
g = torch.Generator().manual_seed(0)
qkv = (torch.randn(B, T, 3 * H * HD, generator=g) * 0.5).cuda().bfloat16()
o, lse = A.attn_fwd(qkv, H)
do = (torch.randn(B, T, H * HD, generator=g) * 0.5).cuda().bfloat16()
for _ in range(5):
    A.attn_bwd(qkv, o, lse, do, H)
torch.cuda.synchronize()
S = 18
nblk = 4 * B * H
buf = np.zeros(4096 * S, dtype=np.uint64)
L = N.lib()
L.dtc_attn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_long]
rc = L.dtc_attn_stamps(buf.ctypes.data, buf.size)
assert rc == 0, f"stamps unavailable (rc {rc}): build with -DDTC_ATTN_STAMPS"
st = buf[:nblk * S].reshape(nblk, S).astype(np.int64)
t0 = st[:, 0].min()
us = (st - t0) / 100.0  # 100 MHz -> us
entry, staged, ends = us[:, 0], us[:, 1], us[:, 2:]
kv, dq = slice(0, 2 * B * H), slice(2 * B * H, nblk)
print(f"kernel span {ends.max():.2f} us")
for name, sl in (("dK/dV", kv), ("dQ", dq)):
    e, s_, en = entry[sl], staged[sl], ends[sl]
    print(f"{name:6s} entry [{e.min():6.2f}, {e.max():6.2f}]  staging {np.median(s_ - e):5.2f} us (max {np.max(s_ - e):5.2f})  "
          f"wave compute median {np.median(en - s_[:, None]):5.2f} max {np.max(en - s_[:, None]):5.2f}  "
          f"block end [{en.max(1).min():6.2f}, {en.max(1).max():6.2f}]")
w = ends[kv] - staged[kv][:, None]
print("dK/dV per-wave compute (median over blocks):", np.round(np.median(w, 0), 2))
w = ends[dq] - staged[dq][:, None]
print("dQ per-wave compute (median over blocks):   ", np.round(np.median(w, 0), 2))
