#!/bin/bash
# GPU-box A/B of library builds / runtime switches on the headline engine step.
# Each config is "label|ENV=val ENV2=val|bench args" (SPECDEC_LIB=libspecdec_x.so selects a `make variant`
# build; bench args e.g. "--option FUSED_VERIFY=0" pick another dispatch path); every config runs
# bench.py --profile-only (B=32 engine step, 5 trials), REPS times, alternating.
# usage: CONFIGS="base||;unfused||--option FUSED_VERIFY=0;pipe8|SPECDEC_LIB=libspecdec_pipe8.so|" [REPS=2] \
#        [TESTS="tests/..."] bash scripts/gpu_ab_bench.sh
set -eo pipefail
R0=$GRAFT_REPO_ROOT
cd $R0
REPS=${REPS:-2}
if [ -n "$TESTS" ]; then
  # the candidate (last config) under the given GPU tests first
  last="${CONFIGS##*;}"
  lenv="${last#*|}"
  env ${lenv%%|*} timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/ab_tests.log 2>&1
fi
IFS=';' read -ra CFG <<< "$CONFIGS"
for rep in $(seq $REPS); do
  for c in "${CFG[@]}"; do
    label="${c%%|*}"
    rest="${c#*|}"
    envs="${rest%%|*}"
    bargs=""
    [[ "$rest" == *"|"* ]] && bargs="${rest#*|}"
    echo -n "$label " >> gpurun_out/ab_bench.txt
    env $envs timeout -k 10 120 python bench.py --profile-only --steps 200 ${BENCH_ARGS} $bargs 2>>gpurun_out/ab_bench.err \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(json.dumps({'ms_per_step': round(d['ms_per_step']*1e3,2), 'trials': [round(t*1e3,2) for t in d['replays']['trial_ms_per_step']], 'draw_in_step': round(k['k_draw']['ms']*1e3,2), 'draw_isolated': round(k['k_draw']['isolated_ms']*1e3,2), 'verify': round(d['phases_ms']['verify']*1e3,2)}))" \
      >> gpurun_out/ab_bench.txt
  done
done
cat gpurun_out/ab_bench.txt
