#!/bin/bash
# GPU-box recipe: instruction-cache PMC pass on a short bench run (counters only, kernel-trace)
set -eo pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv -d $R/gpurun_out/pmc_icache -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 --no-cpu-baseline > $R/gpurun_out/pmc_icache.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc_sq2 -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --prof-steps 5 --no-cpu-baseline > $R/gpurun_out/pmc_sq2.log 2>&1
