#!/bin/bash
# round 4, GPU call AE: closing check of the final defaults -- the whole GPU suite, smoke, 1-GPU bench,
# and multi-rank rehearsals of the driver's benches on this one GPU over gloo (dp2, dp8, tp2, pp2)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4ae_tests.log 2>&1 || { tail -40 gpurun_out/r4ae_tests.log; exit 1; }
tail -2 gpurun_out/r4ae_tests.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ae_smoke.log 2>&1 || { tail -20 gpurun_out/r4ae_smoke.log; exit 1; }
tail -1 gpurun_out/r4ae_smoke.log
$T 300 python bench.py --steps 50 --warmup 5 > gpurun_out/r4ae_bench.log 2>&1 || { tail -30 gpurun_out/r4ae_bench.log; exit 1; }
grep '^{' gpurun_out/r4ae_bench.log | cut -c1-300
port=29561
for cfg in "2 dp" "8 dp" "2 tp" "2 pp"; do
  set -- $cfg
  port=$((port + 1))
  DTC_DIST_BACKEND=gloo $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus $1 --parallel $2 --steps 3 --warmup 2 > gpurun_out/r4ae_$2$1.log 2>&1 || { tail -30 gpurun_out/r4ae_$2$1.log; exit 1; }
  grep '^{' gpurun_out/r4ae_$2$1.log | cut -c1-200
done
