#!/bin/bash
# GPU-box: k_draw launch time for every library variant in LIBS x draw-stage setting in STAGES
# x extra environment in ENVS (scripts/draw_bench.py; SD_DRAW_STAGES picks the span length)
set -eo pipefail
cd $GRAFT_REPO_ROOT
for l in ${LIBS:-libspecdec.so}; do
  for st in ${STAGES:-0}; do
    for e in ${ENVS:-NONE=1}; do
      if [ "$st" = "0" ]; then unset SD_DRAW_STAGES; else export SD_DRAW_STAGES=$st; fi
      echo -n "stages=$st $e " >> gpurun_out/draw_ab.txt
      env $e SPECDEC_LIB=$l timeout -k 10 120 python scripts/draw_bench.py 2>/dev/null >> gpurun_out/draw_ab.txt
    done
  done
done
