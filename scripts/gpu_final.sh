#!/bin/bash
# Short GPU-box recipe for a round's last check: GPU tests, smoke, the default bench line and a
# rocprofv3 kernel-trace summary of the bench's engine step.  Outputs under gpurun_out/.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 100 --no-cpu-baseline --no-configs1 --stream-steps 0 > $R/gpurun_out/prof.log 2>&1
