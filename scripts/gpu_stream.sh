#!/bin/bash
# GPU-box recipe: the STREAM (bit-exact) path — its GPU tests first, then the engine step's time and
# a rocprofv3 kernel summary of it; ALL=1 runs every GPU test and one bench line first.  Outputs
# under gpurun_out/.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_stream_draw.py tests/test_gpu_mt19937.py tests/test_gpu_parity.py tests/test_gpu_errors.py > gpurun_out/gpu_tests_first.log 2>&1
if [ -n "$ALL" ]; then
  timeout -k 10 600 $T tests/ > gpurun_out/gpu_tests.log 2>&1
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err
fi
timeout -k 10 120 python scripts/stream_timing.py >> gpurun_out/stream_strides.txt 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stream -o run -- \
  python3 $R/scripts/stream_timing.py > $R/gpurun_out/prof_stream.log 2>&1
if [ -n "$E2E" ]; then
  cd $R && timeout -k 10 400 python scripts/e2e_timing.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err
fi
