#!/bin/bash
# GPU-box recipe: A/B of tuning environment settings.  Each line of $1 (default
# scripts/ab_cases.txt) is "<name> <VAR=value ...>"; per case: one bench line and a rocprofv3
# kernel-trace summary (outputs under gpurun_out/ab_<name>*).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
CASES=${1:-scripts/ab_cases.txt}
export TMPDIR=/tmp
while read -r name envs; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  ( cd /tmp && env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_prof_$name -o run -- python3 $R/bench.py --steps 100 --no-cpu-baseline > $R/gpurun_out/ab_prof_$name.log 2>&1 )
done < $CASES
