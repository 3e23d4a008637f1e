"""hipBLASLt (torch.matmul) yardstick for benchmarks/gemm_square_micro.hip: random bf16, same shapes/layouts."""
import torch

for S in (4096, 8192):
    a = torch.rand(S, S, device="cuda", dtype=torch.bfloat16) * 2 - 1
    b = torch.rand(S, S, device="cuda", dtype=torch.bfloat16) * 2 - 1
    for name, f in (("NT", lambda: a @ b.t()), ("TN", lambda: a.t() @ b)):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20 if S == 4096 else 5
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(f"torch {S}^3 {name}: {us:.1f} us {2 * S ** 3 / us / 1e6:.0f} TF/s", flush=True)
