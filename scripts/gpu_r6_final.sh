#!/bin/bash
# Round-6 closing evidence (GPU box): the whole GPU suite, the default bench line, rocprofv3 kernel
# traces of the B=32 headline step and the B=512 sweep step (--profile-only), their FETCH_SIZE /
# WRITE_SIZE passes, a kernel trace of the pipelined STREAM step and the B = 512 ticket-order phase
# probe (scripts/ticket_phases.py, the timing build).  Outputs under gpurun_out/;
# every GPU step has its own time limit and the first failure ends the script.
#   SKIP_TESTS=1 / SKIP_BENCH=1 skip those steps.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    > gpurun_out/gpu_tests.log 2>&1
  tail -3 gpurun_out/gpu_tests.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  cut -c1-300 gpurun_out/bench.json
fi
export TMPDIR=/tmp
cd /tmp
for B in 32 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b$B -o run -- \
    python3 $R/bench.py --steps 100 --profile-only --batch $B > $R/gpurun_out/prof_b$B.json 2> $R/gpurun_out/prof_b$B.log
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_b${B}_$c -o run -- \
      python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 --profile-only --batch $B \
      > $R/gpurun_out/pmc_b${B}_$c.log 2>&1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stream -o run -- \
  python3 $R/scripts/stream_timing.py > $R/gpurun_out/prof_stream.txt 2> $R/gpurun_out/prof_stream.log
cd $R
timeout -k 10 180 python scripts/ticket_phases.py > gpurun_out/ticket_phases_B512.txt 2>&1
