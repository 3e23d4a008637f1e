#!/bin/bash
# round 4, GPU call R: empty hipGraph segments dropped (StepProgram._cut checks the node count) --
# graph/dist/engine GPU tests, 1-GPU bench, DP2 gloo rehearsal (segment count, no empty-graph warning)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dist_gpu.py tests/test_engine_gpu.py > gpurun_out/r4r_tests.log 2>&1 || { tail -30 gpurun_out/r4r_tests.log; exit 1; }
tail -2 gpurun_out/r4r_tests.log
$T 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r4r_bench.log 2>&1 || { tail -30 gpurun_out/r4r_bench.log; exit 1; }
grep '^{' gpurun_out/r4r_bench.log | cut -c1-400
DTC_DIST_BACKEND=gloo $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 2 > gpurun_out/r4r_dp2.log 2>&1 || { tail -30 gpurun_out/r4r_dp2.log; exit 1; }
grep -c "Graph is empty" gpurun_out/r4r_dp2.log || true
grep '^{' gpurun_out/r4r_dp2.log | grep -o '"graph_segments.*eager_collectives": [0-9]*'
