#!/bin/bash
# round 4, GPU call Z: final defaults (lm_head dgrad 256x192, grouped wgrad tail split)
# -- the whole GPU suite, smoke, 1-GPU bench, kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4z_tests.log 2>&1 || { tail -40 gpurun_out/r4z_tests.log; exit 1; }
tail -2 gpurun_out/r4z_tests.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z_smoke.log 2>&1 || { tail -20 gpurun_out/r4z_smoke.log; exit 1; }
tail -1 gpurun_out/r4z_smoke.log
$T 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r4z_bench.log 2>&1 || { tail -30 gpurun_out/r4z_bench.log; exit 1; }
grep '^{' gpurun_out/r4z_bench.log | cut -c1-300
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_z -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4z_prof.log 2>&1 || { tail -30 gpurun_out/r4z_prof.log; exit 1; }
echo prof done
