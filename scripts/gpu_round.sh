#!/bin/bash
# GPU-box recipe for the round's evidence: GPU tests, the default bench line (with the CPU
# baseline), a rocprofv3 kernel-trace summary and the FETCH_SIZE / WRITE_SIZE PMC passes.
# Outputs under gpurun_out/.  Every GPU step has its own time limit; the first failure ends it.
# SKIP_TESTS=1 skips the pytest step.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 $T tests/ > gpurun_out/gpu_tests.log 2>&1
fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
export TMPDIR=/tmp
cd /tmp
# profiling passes: the engine step only (no CPU baseline, no STREAM / configs[1] extras, whose
# launches of the same kernel families would mix into the per-kernel averages)
X="--no-cpu-baseline --no-configs1 --stream-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 100 $X > $R/gpurun_out/prof.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_$c -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 $X > $R/gpurun_out/pmc_$c.log 2>&1
done
cd $R && timeout -k 10 200 python scripts/ngram_store_timing.py > gpurun_out/ngs_timing.json 2> gpurun_out/ngs_timing.err
