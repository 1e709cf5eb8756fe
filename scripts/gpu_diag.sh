#!/bin/bash
# GPU-box recipe: perf-mode tests + phase timing + short bench (outputs under gpurun_out/)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_perfmode.py -q -m gpu -x -s > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
