#!/bin/bash
# quick GPU check: full GPU tests, the bench line, and a rocprofv3 kernel-trace summary of the bench
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
export TMPDIR=/tmp
cd /tmp
X="--no-cpu-baseline --no-configs1 --stream-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 100 $X > $R/gpurun_out/prof.log 2>&1
