#!/bin/bash
# Round-5 nucleus-draw A/B (GPU box): the draw tests on the new library, the rejection draw's
# phases, and configs[1] step times of HEAD's library (libspecdec_head.so) vs the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b3
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_draw.py tests/test_gpu_errors.py > $O/tests.log 2>&1 &&
THR_NUC=1 timeout -k 10 120 python -u scripts/thr_phases.py > $O/nuc_phases.txt 2>&1 &&
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib timeout -k 10 150 python -u scripts/b1_ab.py "" >> $O/b1_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/b1_ab.txt
done
echo "exit $?"
