#!/bin/bash
# GPU-box recipe: rocprofv3 PMC passes (counters only, kernel-trace) on a short bench run.
set -eo pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
run() {  # $1 = tag, rest = counters
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_$tag -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 --no-cpu-baseline > $R/gpurun_out/pmc_$tag.log 2>&1
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run grbm GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD
