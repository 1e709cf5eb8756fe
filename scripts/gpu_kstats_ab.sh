#!/bin/bash
# GPU-box recipe: k_stats time (roofline kernel_ms) under the structural knobs, bench workload.
set -eo pipefail
cd $GRAFT_REPO_ROOT
run() {  # $1 = tag, rest = env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$tag.json')); r=d['roofline']; print('%-14s k_stats %.2f us  step %.2f us' % ('$tag', r['kernel_ms']*1e3, d['ms_per_step']*1e3))"
}
run base SD_NOTHING=0
run notails SD_TAILS=0
run decsample SD_DEC_IN_SAMPLE=1
run nounroll SD_STATS_UNROLL=0
run st8 SD_STATS_STAGES=8
run st32 SD_STATS_STAGES=32
