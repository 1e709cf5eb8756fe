#!/bin/bash
# GPU-box recipe: the three GPU test files, then the per-config step timing (scripts/config_timing.py).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_parity.py > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 $T tests/test_gpu_perfmode.py tests/test_gpu_draw.py > gpurun_out/gpu_perf_tests.log 2>&1
timeout -k 10 300 python scripts/config_timing.py ${CFG:-cfg1 cfg4} > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_cfg -o run -- \
    python3 $R/scripts/config_timing.py ${CFG:-cfg1 cfg4} > $R/gpurun_out/prof_cfg.log 2>&1
fi
