#!/bin/bash
# Round-5 keep_vec A/B (GPU box): the whole GPU suite on the new library, then configs[1] / [4]
# of HEAD's library vs the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b17
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 &&
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib CFG_NO_CPU=1 timeout -k 10 200 python -u scripts/config_timing.py cfg1 cfg4 >> $O/cfg_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/cfg_ab.txt
done
echo "exit $?"
