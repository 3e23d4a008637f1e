"""Which hipBLASLt kernels torch.matmul picks for the GPT-2 small layer shapes and the 4096^3 / 8192^3 squares.

Run under `rocprofv3 --kernel-trace --stats -- python benchmarks/hipblaslt_kernel_names.py`: the kernel
names encode hipBLASLt's macro tile (MT), MFMA shape, wave group and depth -- the tile/schedule it chose
where it beats our one-round layer GEMMs (profiles/r6_gemm_square.md).  Prints the per-shape time too.
"""
import torch

SHAPES = [  # (name, M, N, K, layout): NT = x @ w.t() (forward / NT dgrad), NN = dy @ w (NN dgrad)
    ("qkv_fwd", 8192, 2304, 768, "NT"),
    ("out_fwd", 8192, 768, 768, "NT"),
    ("fc1_fwd", 8192, 3072, 768, "NT"),
    ("fc2_fwd", 8192, 768, 3072, "NT"),
    ("fc1_dgrad_nt", 8192, 768, 3072, "NT"),
    ("fc2_dgrad_nn", 8192, 3072, 768, "NN"),
    ("sq4096_nt", 4096, 4096, 4096, "NT"),
    ("sq8192_nt", 8192, 8192, 8192, "NT"),
]


def main():
    torch.manual_seed(0)
    for name, M, N, K, lay in SHAPES:
        a = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
        if lay == "NT":
            w = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
            f = lambda: a @ w.t()
        else:
            w = torch.rand(K, N, device="cuda", dtype=torch.bfloat16) * 2 - 1
            f = lambda: a @ w
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(f"{name} [{M}x{N}x{K} {lay}]: {us:.1f} us warm, {2 * M * N * K / us / 1e6:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
