"""Latency of the xGMI P2P all-reduce kernels (parallel/p2p.py) per call, one-shot vs two-shot, at the
TP message sizes, with W ranks: fp32 one-shot / two-shot, and the bf16 payload (tp_comm_dtype: bf16)
staged by a copy kernel vs written in place by its producer (``x=None``: one launch fewer).  On a multi-GPU node this is the real xGMI number; on the 1-GPU dev box
the W processes share one device (IPC within a device), so it measures the kernel path itself —
launches, device barriers, the copy/reduce passes at HBM speed — not link bandwidth.

    python benchmarks/p2p_bench.py [--world 2] [--reps 50] [--json out.json]
"""

import argparse
import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SIZES = [64 << 10, 512 << 10, 1 << 20, 4 << 20, 8 << 20, 25 << 20]  # 25 MB: GPT-2 small [8192, 768] fp32


def _worker(reps, out_dir):
    os.environ.setdefault("DTC_DIST_BACKEND", "gloo")
    import torch.distributed as dist

    from distributed_training_compare_jax_amd.parallel.dist import destroy, init_distributed
    from distributed_training_compare_jax_amd.parallel.p2p import P2PAllReduce

    d = init_distributed("cuda")
    ar = P2PAllReduce(dist.group.WORLD, d.rank, d.world, d.device, max(SIZES))
    res = {}
    for nbytes in SIZES:
        n = nbytes // 4
        t = torch.full((n,), float(d.rank + 1), device=d.device)
        xb = torch.full((n,), float(d.rank + 1), dtype=torch.bfloat16, device=d.device)
        ob = torch.empty(n, device=d.device)
        variants = [(2, "one-shot", lambda m: ar.all_reduce_(t, mode=m)), (1, "two-shot", lambda m: ar.all_reduce_(t, mode=m)),
                    # tp_comm_dtype: bf16 (the same element count, half the bytes): copied into the buffer
                    # by the stage kernel, or already written there by its producer GEMM (staged)
                    (0, "bf16 copy", lambda m: ar.all_reduce_bf16(xb, ob, mode=m)),
                    (0, "bf16 staged", lambda m: ar.all_reduce_bf16(None, ob, mode=m))]
        for mode, name, call in variants:
            if mode == 2 and nbytes > (8 << 20):
                continue
            # captured: reps calls in one hipGraph (how the step runs them), timed by events
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                g.capture_begin(capture_error_mode="thread_local")
                for _ in range(reps):
                    call(mode)
                ar.end_step()
                g.capture_end()
            torch.cuda.current_stream().wait_stream(s)
            times = []
            for _ in range(3):
                t.fill_(float(d.rank + 1))
                torch.cuda.synchronize()
                dist.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                times.append(e0.elapsed_time(e1) * 1e3 / reps)
            ar.check()
            res[f"{name} {nbytes >> 10} KB"] = min(times)
            del g
    torch.save(res, os.path.join(out_dir, f"r{d.rank}.pt"))
    ar.close()
    destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from distributed_training_compare_jax_amd.parallel.dist import spawn

    with tempfile.TemporaryDirectory() as td:
        spawn(_worker, a.world, args=(a.reps, td))
        r = [torch.load(os.path.join(td, f"r{i}.pt")) for i in range(a.world)]
    ndev = torch.cuda.device_count()
    print(f"P2P all-reduce, W={a.world} ranks on {min(ndev, a.world)} device(s): us per call (captured, min of 3)")
    out = {}
    for k in r[0]:
        v = max(x[k] for x in r)
        out[k] = v
        print(f"  {k:24s} {v:8.1f} us")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
