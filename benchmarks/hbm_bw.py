"""Achievable HBM bandwidth on this GPU (the ceiling for the memory-bound step kernels: LayerNorm, AdamW,
CE backward, casts): device-to-device copy, write-only fill and read-mostly sum at several sizes, timed with
events over graph-replayed repetitions.

    python benchmarks/hbm_bw.py
"""
import torch


def gtime(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        for _ in range(reps):
            fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    for mb in (64, 256, 1024):
        n = mb * (1 << 20) // 4
        a = torch.empty(n, device="cuda")
        b = torch.empty(n, device="cuda")
        a.fill_(1.0)
        t = gtime(lambda: b.copy_(a))
        print(f"copy  {mb:5d} MB: {2 * a.numel() * 4 / t / 1e12:5.2f} TB/s (read + write)", flush=True)
        t = gtime(lambda: b.fill_(2.0))
        print(f"fill  {mb:5d} MB: {b.numel() * 4 / t / 1e12:5.2f} TB/s (write)", flush=True)
        out = torch.empty((), device="cuda")
        t = gtime(lambda: torch.sum(a, dim=0, out=out))
        print(f"sum   {mb:5d} MB: {a.numel() * 4 / t / 1e12:5.2f} TB/s (read)", flush=True)
        del a, b


if __name__ == "__main__":
    main()
