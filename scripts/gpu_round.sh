#!/bin/bash
# GPU-box recipe for the round's evidence: GPU tests, the default bench line (with the CPU
# baseline), a rocprofv3 kernel-trace summary and the FETCH_SIZE / WRITE_SIZE PMC passes.
# Outputs under gpurun_out/.  Every GPU step has its own time limit; the first failure ends it.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 100 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_$c -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 --no-cpu-baseline > $R/gpurun_out/pmc_$c.log 2>&1
done
cd $R && timeout -k 10 200 python scripts/ngram_store_timing.py > gpurun_out/ngs_timing.json 2> gpurun_out/ngs_timing.err
