#!/bin/bash
# GPU-box recipe: parity + perf tests, then A/B of perf-mode structure (SD_TAILS=1 tails vs 0
# own launches): rocprof + bench for each (outputs under gpurun_out/)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x > gpurun_out/gpu_perf_tests.log 2>&1
SD_TAILS=0 timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x > gpurun_out/gpu_perf_tests_t0.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
export TMPDIR=/tmp
for t in 1 0; do
  ( cd /tmp && SD_TAILS=$t timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_t$t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_t$t.log 2>&1 )
  SD_TAILS=$t timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_t$t.json 2> gpurun_out/bench_t$t.err
done
