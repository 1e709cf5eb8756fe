#!/bin/bash
# GPU-box recipe for a kernel change: the new / named test files first (fast failure), every GPU
# test, one bench line, a rocprofv3 kernel summary.  FIRST="tests/x.py ..." names the first files.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
if [ -n "$FIRST" ]; then
  timeout -k 10 300 $T $FIRST > gpurun_out/gpu_tests_first.log 2>&1
fi
timeout -k 10 600 $T tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_check -o run -- \
  python3 $R/bench.py --steps 100 --no-cpu-baseline > $R/gpurun_out/prof_check.log 2>&1
