#!/bin/bash
# GPU-box recipe: perf-mode + parity tests, then the k_stats / step A/B and the phase timing
set -eo pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_perfmode.py tests/test_gpu_draw.py > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_gpu_threshold.py > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 bash scripts/gpu_kstats_ab.sh > gpurun_out/kab.txt 2>&1
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase.log 2>&1
