#!/bin/bash
# GPU-box recipe: all GPU tests, bench, rocprof summary, phase timing (outputs under gpurun_out/)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase.log 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
