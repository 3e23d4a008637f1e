"""Does a replayed hipGraph run two independent captured branches concurrently?  Captures a
main-stream chain and a side-stream chain (blocked or interleaved capture order) and compares the
replay time with the serial sum.  Prints one line per variant."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import gemm as G  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
r = lambda *s: (torch.randn(*s, generator=g) * 0.1).to(dev).to(torch.bfloat16)
xa, wa = r(4096, 512), r(512, 512)
xb, wb = r(4096, 512), r(512, 512)
ya = torch.empty(4096, 512, device=dev, dtype=torch.bfloat16)
G.reserve_workspace(dev, 64 << 20)
G.reserve_workspace(dev, 64 << 20, role="side")
N = 12


def chain(x, w):
    y = x
    for _ in range(N):
        y = G.linear(y, w, None)
    return y


def timed(fn, reps=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def capture(order):
    side = torch.cuda.Stream()
    cap = torch.cuda.Stream()
    gr = torch.cuda.CUDAGraph()
    keep = []
    with torch.cuda.stream(cap):
        gr.capture_begin(capture_error_mode="thread_local")
        side.wait_stream(cap)
        if order == "blocked":
            keep.append(chain(xa, wa))
            with torch.cuda.stream(side), G.workspace_role("side"):
                keep.append(chain(xb, wb))
        else:  # interleaved
            ya_, yb_ = xa, xb
            for _ in range(N):
                ya_ = G.linear(ya_, wa, None)
                with torch.cuda.stream(side), G.workspace_role("side"):
                    yb_ = G.linear(yb_, wb, None)
            keep += [ya_, yb_]
        cap.wait_stream(side)
        gr.capture_end()
    return gr, keep


one = timed(lambda: chain(xa, wa))
print(f"eager single chain      {one:8.1f} us")
for order in ("blocked", "interleaved"):
    gr, keep = capture(order)
    t = timed(gr.replay)
    print(f"graph 2 chains {order:11s} {t:8.1f} us  (serial would be ~{2 * one:.0f})")
