#!/bin/bash
# Round-6 large-batch A/B (GPU box): the given GPU tests on the candidate library, then the headline
# step and bench.py's sweep for each library / option set, and the ticket-order phase probe.
#   TESTS="tests/..."          pytest -m gpu targets ("" skips); PYTEST_K="expr" adds -k "expr"
#   LIBS="old new"             libraries: "new" = libspecdec.so, else libspecdec_<name>.so
#   SWEEP_CONFS='"" "SAMP_CHUNKS=2"'   sd_set_option sets for the candidate's sweep (scripts/sweep_ab.py)
#   SWEEP_B="128,512"          batches of the sweep
#   PHASES_B="512"             scripts/ticket_phases.py batches ("" skips; needs `make timing`)
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
LIBS=${LIBS:-"old new"}
SWEEP_B=${SWEEP_B:-"128,512"}
if [ -n "$TESTS" ]; then
  KARGS=()
  [ -n "$PYTEST_K" ] && KARGS=(-k "$PYTEST_K")
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "${KARGS[@]}" $TESTS \
    > gpurun_out/ab_tests.log 2>&1
  tail -2 gpurun_out/ab_tests.log
fi
libfile() { if [ "$1" = new ]; then echo libspecdec.so; else echo libspecdec_$1.so; fi; }
CONFIGS=""
for L in $LIBS; do CONFIGS="$CONFIGS;$L|SPECDEC_LIB=$(libfile $L)|"; done
CONFIGS="${CONFIGS#;}" REPS=${REPS:-2} bash scripts/gpu_ab_bench.sh
for L in $LIBS; do
  if [ "$L" = new ]; then
    eval "set -- $SWEEP_CONFS"
    [ $# -eq 0 ] && set -- ""
  else
    set -- ""
  fi
  echo "== $L" >> gpurun_out/ab_sweep.txt
  SPECDEC_LIB=$(libfile $L) timeout -k 10 300 python scripts/sweep_ab.py $SWEEP_B "$@" >> gpurun_out/ab_sweep.txt
done
cat gpurun_out/ab_sweep.txt
for B in $PHASES_B; do
  B=$B timeout -k 10 180 python scripts/ticket_phases.py > gpurun_out/ticket_phases_B$B.txt 2>&1
done
