"""Backward-like schedule (per layer: a main-stream chain, then side-stream work that depends on
it): single hipGraph with a fork per layer vs two graphs (main / side) on two streams synchronised
by device-side flag kernels (ops: dtc_flag_set / dtc_flag_wait) vs serial vs main-only."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_compare_jax_amd.ops import _native as N  # noqa: E402
from distributed_training_compare_jax_amd.ops import gemm as G  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
r = lambda *s: (torch.randn(*s, generator=g) * 0.05).to(dev).to(torch.bfloat16)
L, NM, NS = 12, 5, 4
x0 = r(4096, 512)
wm = [r(512, 512) for _ in range(NM)]
xs = r(4096, 512)
ws = [r(512, 512) for _ in range(NS)]
dW = torch.zeros(512, 512, device=dev)
G.reserve_workspace(dev, 64 << 20)
G.reserve_workspace(dev, 64 << 20, role="side")
lib = N.lib()
flags_ms = torch.zeros(64, dtype=torch.int32, device=dev)
flags_sm = torch.zeros(64, dtype=torch.int32, device=dev)
ep_m = torch.zeros(1, dtype=torch.int32, device=dev)
ep_s = torch.zeros(1, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
S = torch.cuda.Stream()
M = torch.cuda.Stream()
keep = []


def main_layer(x):
    for w in wm:
        x = G.linear(x, w, None)
    return x


def side_layer(x):
    for w in ws:
        G.wgrad(x, xs, dW, 1.0)   # dW += x^T xs  (a weight-gradient-shaped GEMM)


def sp(t):
    return N.stream_ptr(dev)


def run_single(mode):
    x = x0
    for l in range(L):
        x = main_layer(x)
        if mode == "fork":
            S.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(S), G.workspace_role("side"):
                side_layer(x)
            keep.append(x)
        elif mode == "serial":
            side_layer(x)
    if mode == "fork":
        torch.cuda.current_stream().wait_stream(S)
    return x


def capture_single(mode):
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(M):
        gr.capture_begin(capture_error_mode="thread_local")
        run_single(mode)
        gr.capture_end()
    return gr


def capture_dual():
    gm, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(M):
        gm.capture_begin(capture_error_mode="relaxed")
    with torch.cuda.stream(S):
        gs.capture_begin(capture_error_mode="relaxed")
        N.check(lib.dtc_epoch_inc(ep_s.data_ptr(), N.stream_ptr(dev)), "epoch")
    with torch.cuda.stream(M):
        N.check(lib.dtc_epoch_inc(ep_m.data_ptr(), N.stream_ptr(dev)), "epoch")
    x = x0
    for l in range(L):
        with torch.cuda.stream(M):
            x = main_layer(x)
            keep.append(x)
            N.check(lib.dtc_flag_set(flags_ms.data_ptr(), l, ep_m.data_ptr(), N.stream_ptr(dev)), "set")
        with torch.cuda.stream(S), G.workspace_role("side"):
            N.check(lib.dtc_flag_wait(flags_ms.data_ptr(), l, ep_s.data_ptr(), err.data_ptr(), N.stream_ptr(dev)), "wait")
            side_layer(x)
    with torch.cuda.stream(S):
        N.check(lib.dtc_flag_set(flags_sm.data_ptr(), 0, ep_s.data_ptr(), N.stream_ptr(dev)), "set")
        gs.capture_end()
    with torch.cuda.stream(M):
        N.check(lib.dtc_flag_wait(flags_sm.data_ptr(), 0, ep_m.data_ptr(), err.data_ptr(), N.stream_ptr(dev)), "wait")
        gm.capture_end()
    return gm, gs


def timed(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


res = {}
for mode in ("mainonly", "serial", "fork"):
    gr = capture_single(mode)
    res[mode] = timed(lambda: gr.replay())
gm, gs = capture_dual()


def dual():
    with torch.cuda.stream(S):
        gs.replay()
    with torch.cuda.stream(M):
        gm.replay()


res["dual"] = timed(dual)
torch.cuda.synchronize()
print({k: round(v, 1) for k, v in res.items()}, "err", int(err.item()))
