#!/bin/bash
# GPU-box recipe: parity + perf-mode tests, then bench + rocprofv3 kernel-trace summary
# (outputs under gpurun_out/)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x -s > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
