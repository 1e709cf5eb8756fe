#!/bin/bash
# GPU-box recipe: smoke, bench, rocprofv3 kernel-trace summary (outputs under gpurun_out/)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
