#!/bin/bash
# round 4, GPU call AJ: after deleting the measured-slower variants (qkv K-split tail, 256x192 qkv forward,
# bf16 dgrad outputs, delta epilogue) -- the whole GPU suite, smoke, 1-GPU bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4aj_tests.log 2>&1 || { tail -40 gpurun_out/r4aj_tests.log; exit 1; }
tail -2 gpurun_out/r4aj_tests.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4aj_smoke.log 2>&1 || { tail -20 gpurun_out/r4aj_smoke.log; exit 1; }
tail -1 gpurun_out/r4aj_smoke.log
$T 300 python bench.py --steps 50 --warmup 5 > gpurun_out/r4aj_bench.log 2>&1 || { tail -30 gpurun_out/r4aj_bench.log; exit 1; }
grep '^{' gpurun_out/r4aj_bench.log | cut -c1-300
