#!/bin/bash
# Round-5 batch-1 lean-verify A/B (GPU box): the lean / fused / parity tests on the new library,
# phase timings, and configs[1] step times of HEAD's library (libspecdec_mtold.so), the
# decide-only change (libspecdec_pair.so) and the row-wave prologue (libspecdec.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b2
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_lean_verify.py tests/test_gpu_parity.py tests/test_gpu_threshold.py tests/test_gpu_errors.py > $O/tests.log 2>&1 &&
B=1 RULE=spec timeout -k 10 120 python -u scripts/phase_timing.py > $O/lean_phases.txt 2>&1 &&
for lib in libspecdec_mtold.so libspecdec_pair.so libspecdec.so libspecdec_mtold.so libspecdec_pair.so libspecdec.so; do
    SPECDEC_LIB=$lib timeout -k 10 150 python -u scripts/b1_ab.py "" >> $O/b1_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/b1_ab.txt
done
echo "exit $?"
