#!/bin/bash
# Round-5 lean-verify dynamic-LDS A/B (GPU box): lean / parity / perfmode tests on the new library,
# then the shard lines (16 / 8 / 4 rows) and configs[1] of HEAD's library vs the new one (and the
# new one with the lean verify forced for <= 8 sequences).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b9
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_lean_verify.py tests/test_gpu_parity.py tests/test_gpu_perfmode.py tests/test_gpu_errors.py \
    > $O/tests.log 2>&1 &&
B="python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --stream-steps 0 --no-e2e --trials 3"
for run in "libspecdec_head.so|" "libspecdec.so|" "libspecdec.so|--option LEAN_VERIFY=1" "libspecdec_head.so|" "libspecdec.so|"; do
    lib=${run%%|*}; opt=${run#*|}
    SPECDEC_LIB=$lib timeout -k 10 300 $B $opt > $O/tmp.json 2>> $O/bench.err || exit 1
    python - "$lib $opt" $O/tmp.json >> $O/ab.txt <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], round(d["ms_per_step"] * 1e3, 2),
              {k: round(v["ms_per_step"] * 1e3, 2) for k, v in d["shard_rows"].items()},
              {k: round(v["us_per_step"], 2) for k, v in d["configs1"].items()}, round(d["configs4"]["us_per_step"], 2))
PY
done
echo "exit $?"
