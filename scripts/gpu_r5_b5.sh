#!/bin/bash
# Round-5 threshold A/B (GPU box): threshold / parity / draw / lean tests on the new library, the
# 9-row threshold phases, and configs[1] step times of HEAD's library vs the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_threshold.py tests/test_gpu_parity.py tests/test_gpu_draw.py tests/test_gpu_lean_verify.py \
    tests/test_gpu_errors.py > $O/tests.log 2>&1 &&
THR_ROWS=9 timeout -k 10 120 python -u scripts/thr_phases.py > $O/thr_phases_9.txt 2>&1 &&
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib timeout -k 10 150 python -u scripts/b1_ab.py "" >> $O/b1_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/b1_ab.txt
done
echo "exit $?"
