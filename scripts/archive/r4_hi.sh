#!/bin/bash
# round 4, GPU calls H + I together: P2P v3 multi-rank tests and bench, attention A/B (rescale kept a
# branch), cold-cache layer-GEMM A/B
set -u
bash scripts/r4_i.sh || exit $?
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" > gpurun_out/r4hi_attn_tests.log 2>&1 || { tail -20 gpurun_out/r4hi_attn_tests.log; exit 1; }
tail -1 gpurun_out/r4hi_attn_tests.log
timeout -k 10 240 python benchmarks/attn_ab.py --rounds 5 2>&1 | grep -v amdgpu | tee gpurun_out/r4hi_attn_ab.log || exit 1
bash scripts/r4_h.sh
