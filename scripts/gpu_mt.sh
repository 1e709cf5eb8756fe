#!/bin/bash
# GPU-box recipe: the device mt19937 generator — its tests, a stride sweep of the generator alone,
# the STREAM engine step at a few strides, and a rocprofv3 kernel summary.  Outputs under gpurun_out/.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_mt19937.py tests/test_gpu_stream_draw.py > gpurun_out/gpu_tests_mt.log 2>&1
timeout -k 10 200 python scripts/mt_timing.py > gpurun_out/mt_sweep.txt 2>&1
for s in 131072 196608 262144; do
  SPECDEC_MT_STRIDE=$s timeout -k 10 120 python scripts/stream_timing.py >> gpurun_out/stream_strides.txt 2>&1
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stream -o run -- \
  python3 $R/scripts/stream_timing.py > $R/gpurun_out/prof_stream.log 2>&1
