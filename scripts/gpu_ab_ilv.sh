#!/bin/bash
# GPU-box recipe: tests, then bench with interleaved vs contiguous k_stats stages
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
for a in 1 0 1 0; do
  SD_STATS_INTERLEAVE=$a timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 --prof-steps 20 >> gpurun_out/bench_i$a.jsonl 2>/dev/null
done
