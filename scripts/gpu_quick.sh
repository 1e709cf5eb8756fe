#!/bin/bash
# GPU-box quick check: the draw / perf-mode / parity tests (QT overrides the list), then one bench
# line without the CPU baseline.  Outputs under gpurun_out/.
set -eo pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $T ${QT:-tests/test_gpu_draw.py tests/test_gpu_perfmode.py tests/test_gpu_parity.py} > gpurun_out/gpu_quick_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
