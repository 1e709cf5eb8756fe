#!/bin/bash
# GPU-box recipe: instruction counters of configs[1]'s batch-1 kernels (k_draw_lean, the verify),
# one rocprofv3 --pmc pass each, plus a kernel-trace summary.  Outputs under gpurun_out/.
set -eo pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/b1pmc1 -o run -- \
  python3 $R/scripts/b1_verify_loop.py > $R/gpurun_out/b1pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/b1trace -o run -- \
  python3 $R/scripts/b1_verify_loop.py > $R/gpurun_out/b1trace.log 2>&1
