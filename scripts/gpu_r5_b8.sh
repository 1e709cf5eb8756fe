#!/bin/bash
# Round-5 n-gram verify A/B (GPU box): n-gram tests on the new library, configs[4] step times of
# HEAD's library vs the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_ngram_store.py tests/test_gpu_parity.py tests/test_gpu_errors.py > $O/tests.log 2>&1 &&
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib CFG_NO_CPU=1 timeout -k 10 150 python -u scripts/config_timing.py cfg4 >> $O/cfg4_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/cfg4_ab.txt
done
echo "exit $?"
