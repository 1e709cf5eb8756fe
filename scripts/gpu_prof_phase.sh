#!/bin/bash
# GPU-box recipe: phase timing + rocprofv3 kernel summary of the bench (outputs under gpurun_out/)
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase.log 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
