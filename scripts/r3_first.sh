set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3a_bench_ref.log 2>&1 && \
timeout -k 10 300 python bench.py --model gpt2-small --steps 20 --warmup 5 > gpurun_out/r3a_bench_g2s.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --set dtype=fp32 > gpurun_out/r3a_bench_fp32.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a_prof_g2s -o prof --output-format csv -- python bench.py --model gpt2-small --steps 10 --warmup 3 > gpurun_out/r3a_prof_g2s.log 2>&1
echo rc=$?
