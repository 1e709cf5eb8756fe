#!/bin/bash
# GPU-box recipe for the round's evidence: GPU tests, the default bench line (with the CPU
# baseline), a rocprofv3 kernel-trace summary and the FETCH_SIZE / WRITE_SIZE PMC passes.
# Outputs under gpurun_out/.  Every GPU step has its own time limit; the first failure ends it.
# SKIP_TESTS=1 skips the pytest step; SKIP_BENCH=1 the default bench line.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 $T tests/ > gpurun_out/gpu_tests.log 2>&1
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
fi
export TMPDIR=/tmp
cd /tmp
# profiling passes: --profile-only runs the B=32 engine step alone (no shards, configs[1] / [4],
# STREAM or CPU lines), so every sd:: launch has the headline shape; the kernel trace is kept too
# (scripts/trace_summary.py splits it by grid and predecessor)
X="--profile-only"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 100 $X > $R/gpurun_out/prof.json 2> $R/gpurun_out/prof.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_$c -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 $X > $R/gpurun_out/pmc_$c.log 2>&1
done
if [ -z "$SKIP_NGS" ]; then
  cd $R && timeout -k 10 200 python scripts/ngram_store_timing.py > gpurun_out/ngs_timing.json 2> gpurun_out/ngs_timing.err
fi
