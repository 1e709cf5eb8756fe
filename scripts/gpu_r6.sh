#!/bin/bash
# Round-6 GPU recipe, parametrised by environment (every GPU step under its own time limit; the
# first failure ends the script):
#   TESTS="tests/"        pytest -m gpu targets ("" skips)
#   BENCH="..."           bench.py arguments of the full line ("skip" skips)
#   PROF_B="512"          rocprofv3 kernel-trace of `bench.py --profile-only --batch B` ("" skips)
#   PMC_B="512"           FETCH_SIZE / WRITE_SIZE passes of the same ("" skips)
#   EXTRA="cmd"           one more command (A/B scripts), run last under a 300 s limit
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/gpu_tests.log 2>&1
  tail -3 gpurun_out/gpu_tests.log
fi
if [ "$BENCH" != "skip" ]; then
  timeout -k 10 400 python bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.err
  cut -c1-400 gpurun_out/bench.json
fi
export TMPDIR=/tmp
for B in $PROF_B; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b$B -o run -- \
    python3 $R/bench.py --steps 40 --profile-only --batch $B > $R/gpurun_out/prof_b$B.json 2> $R/gpurun_out/prof_b$B.log)
done
for B in $PMC_B; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_b${B}_$c -o run -- \
      python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 --profile-only --batch $B > $R/gpurun_out/pmc_b${B}_$c.log 2>&1)
  done
done
if [ -n "$EXTRA" ]; then
  timeout -k 10 300 bash -c "$EXTRA"
fi
