#!/bin/bash
# Round-5 closing run (GPU box): the whole GPU suite, configs[1] / [4] of the previous library vs
# the current one, then the round's evidence (gpu_round.sh without its test step).  Any failure ends it.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b17
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
cp $O/tests.log gpurun_out/gpu_tests.log
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib CFG_NO_CPU=1 timeout -k 10 200 python -u scripts/config_timing.py cfg1 cfg4 >> $O/cfg_ab.txt 2>&1
    echo "^ $lib" >> $O/cfg_ab.txt
done
SKIP_TESTS=1 bash scripts/gpu_round.sh
echo "final done"
