#!/bin/bash
# GPU-box recipe: all GPU tests, then 3 short benches (outputs under gpurun_out/)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rm -f gpurun_out/bench3.jsonl
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 --prof-steps 20 >> gpurun_out/bench3.jsonl 2>/dev/null
done
