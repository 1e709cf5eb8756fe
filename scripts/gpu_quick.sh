#!/bin/bash
# GPU-box quick check: the draw tests, then one bench line.  Outputs under gpurun_out/.
set -eo pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_draw.py > gpurun_out/gpu_draw_tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
