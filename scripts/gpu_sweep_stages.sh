#!/bin/bash
# GPU-box recipe: tests, then bench ms/step for several k_stats span sizes (SD_STATS_STAGES)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
for st in 0 1 2 3 4 6 12; do
  if [ $st = 0 ]; then unset SD_STATS_STAGES; else export SD_STATS_STAGES=$st; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 --prof-steps 5 > gpurun_out/sweep_$st.json 2>/dev/null
done
