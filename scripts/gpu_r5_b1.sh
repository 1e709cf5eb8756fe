#!/bin/bash
# Round-5 batch-1 / STREAM diagnostics (GPU box): the row-shard test, phase timings of the
# nucleus rejection draw and of the batch-1 lean verify (default and paired-row variant), a
# kernel trace of configs[1], a configs[1] A/B of the variant library, and the STREAM step's
# phases.  Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_mt19937.py tests/test_gpu_lean_verify.py tests/test_gpu_fused.py \
    "tests/test_gpu_perfmode.py::test_batches_beyond_one_call_are_row_sharded" > $O/shard_test.log 2>&1 &&
for lib in libspecdec.so libspecdec_mtold.so libspecdec.so libspecdec_mtold.so; do
    SPECDEC_LIB=$lib STRIDES=65536,131072,196608 timeout -k 10 120 python -u scripts/mt_timing.py >> $O/mt_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/mt_ab.txt
done &&
THR_NUC=1 timeout -k 10 120 python -u scripts/thr_phases.py > $O/nuc_phases.txt 2>&1 &&
B=1 RULE=spec timeout -k 10 120 python -u scripts/phase_timing.py > $O/lean_phases.txt 2>&1 &&
SPECDEC_LIB=libspecdec_pairts.so B=1 RULE=spec timeout -k 10 120 python -u scripts/phase_timing.py > $O/lean_phases_pair.txt 2>&1 &&
for lib in libspecdec_mtold.so libspecdec.so libspecdec_pair.so libspecdec_mtold.so libspecdec.so libspecdec_pair.so; do
    SPECDEC_LIB=$lib timeout -k 10 150 python -u scripts/b1_ab.py "" >> $O/b1_ab.txt 2>&1 || exit 1
    echo "^ $lib" >> $O/b1_ab.txt
done &&
(cd /tmp && export TMPDIR=/tmp CFG_NO_CPU=1 &&
 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_cfg1" -o run \
     -- python3 "$GRAFT_REPO_ROOT/scripts/config_timing.py" cfg1 > "$GRAFT_REPO_ROOT/$O/prof_cfg1.log" 2>&1) &&
timeout -k 10 200 python -u scripts/stream_phases.py > $O/stream_phases.txt 2>&1
echo "exit $?"
