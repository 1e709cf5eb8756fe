#!/bin/bash
# rocprofv3 kernel stats of configs[1] (scripts/config_timing.py cfg1) for each library variant
# named on the command line ("base" = libspecdec.so); GPU box, diagnostic
set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  lib=libspecdec_$v.so
  [ "$v" = base ] && lib=libspecdec.so
  SPECDEC_LIB=$lib CFG_NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/prof_$v -o run -- python3 $R/scripts/config_timing.py cfg1 > $R/gpurun_out/prof_$v.log 2>&1 || exit 1
done
