"""Probe: does a stream forked into a hipGraph capture (s2.wait_stream(capturing)) report itself as
capturing, and can a one-rank RCCL collective be issued from it?  (Round-6 root cause of the bf16 DP chain
crash: ProcessGroupNCCL's watchdog queried an event recorded in a capturing stream.)

    python benchmarks/capture_side_stream_probe.py status|a2a_main|a2a_side"""
import os
import sys

import torch
import torch.distributed as dist

mode = sys.argv[1]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
if mode != "status":
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
x = torch.ones(1 << 16, device=dev, dtype=torch.bfloat16)
y = torch.empty_like(x)
if mode != "status":
    dist.all_to_all_single(y, x)  # eager warmup (communicator init)
torch.cuda.synchronize()
s = torch.cuda.Stream(dev)
s2 = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream(dev))
g = torch.cuda.CUDAGraph()
res = {}
with torch.cuda.stream(s):
    g.capture_begin()
    res["main"] = torch.cuda.is_current_stream_capturing()
    x.mul_(1.0)
    s2.wait_stream(s)
    with torch.cuda.stream(s2):
        res["side_before_work"] = torch.cuda.is_current_stream_capturing()
        x.mul_(1.0)
        res["side_after_work"] = torch.cuda.is_current_stream_capturing()
        if mode == "a2a_side":
            dist.all_to_all_single(y, x)
    s.wait_stream(s2)
    if mode == "a2a_main":
        dist.all_to_all_single(y, x)
    g.capture_end()
torch.cuda.current_stream(dev).wait_stream(s)
print(mode, res, flush=True)
g.replay()
torch.cuda.synchronize()
import time
time.sleep(2.0)  # let the PG watchdog poll any enqueued work
print(mode, "replayed ok", bool(torch.equal(y, x)), flush=True)
os._exit(0)  # (destroy_process_group after a captured collective hung in the round-6 probe)
