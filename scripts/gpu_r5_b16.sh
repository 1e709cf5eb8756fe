#!/bin/bash
# Round-5 threshold dump-sum A/B (GPU box): threshold / parity / draw / lean / errors tests on the
# new library, the 9-row threshold phases, configs[1] and configs[4] of HEAD's library vs the new.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b16
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_threshold.py tests/test_gpu_parity.py tests/test_gpu_draw.py tests/test_gpu_lean_verify.py \
    tests/test_gpu_errors.py tests/test_gpu_perfmode.py > $O/tests.log 2>&1 &&
THR_ROWS=9 timeout -k 10 120 python -u scripts/thr_phases.py > $O/thr_phases_9.txt 2>&1 &&
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib CFG_NO_CPU=1 timeout -k 10 200 python -u scripts/config_timing.py cfg1 cfg4 >> $O/cfg_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/cfg_ab.txt
done
echo "exit $?"
