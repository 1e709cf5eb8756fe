#!/bin/bash
# Round-5 k_resample 8 waves A/B (GPU box): the whole GPU suite on the new library, then the STREAM
# engine step of HEAD's library vs the new one (the tokens checksums must agree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b21
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 &&
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib timeout -k 10 200 python -u scripts/stream_ab.py >> $O/stream_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/stream_ab.txt
done
echo "exit $?"
