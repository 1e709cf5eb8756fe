#!/bin/bash
# GPU-box diagnostics of the STREAM path: the mt19937 round microbenchmark and the phase timelines
# of k_rowsample / k_walk (timing build).  Outputs under gpurun_out/.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 ./scripts/microbench/mt_gen_bench > gpurun_out/mt_gen_bench.txt 2>&1
timeout -k 10 120 python scripts/stream_phases.py > gpurun_out/stream_phases.txt 2>&1
