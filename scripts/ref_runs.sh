# Reference-length runs (5000 timed steps, same YAMLs) on the visible GPUs -> gpurun_out/outputs/<strategy>/
set -e
for s in dp tp pp; do
  timeout -k 10 600 python main.py --train_config_path configs/train_config_$s.yaml --log_every 500 \
      --output_dir gpurun_out/outputs/$s > gpurun_out/main_$s.log 2>&1
  tail -3 gpurun_out/main_$s.log
done
timeout -k 10 300 python bench.py --model gpt2-medium --steps 20 --warmup 3 > gpurun_out/bench_medium.log 2>&1
tail -1 gpurun_out/bench_medium.log
