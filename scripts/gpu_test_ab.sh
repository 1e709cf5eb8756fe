#!/bin/bash
# GPU-box recipe: GPU tests on the default library, the A/B cases, then phase timing
set -eo pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_draw.py tests/test_gpu_perfmode.py > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 600 $T tests/test_gpu_parity.py > gpurun_out/gpu_tests.log 2>&1
bash scripts/gpu_ab_env.sh ${1:-scripts/ab_cases.txt}
bash scripts/gpu_phase2.sh
