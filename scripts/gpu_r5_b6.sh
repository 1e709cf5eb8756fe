#!/bin/bash
# Round-5 STREAM k_walk A/B (GPU box): STREAM tests on the new library, k_walk phases, and the
# STREAM engine step (bench.py --only stream) of HEAD's library vs the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b6
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_engine_surface.py tests/test_gpu_errors.py tests/test_gpu_stream_draw.py \
    > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/stream_phases.py > $O/stream_phases.txt 2>&1 &&
for lib in libspecdec_head.so libspecdec.so libspecdec_head.so libspecdec.so; do
    SPECDEC_LIB=$lib timeout -k 10 200 python -u scripts/stream_ab.py >> $O/stream_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/stream_ab.txt
done
echo "exit $?"
