#!/bin/bash
# Round-5 batch-1 diagnostics (GPU box): draw phases at one row, the threshold search's phases
# (9 rows, the nucleus verify's), a kernel trace of configs[1] on the current library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b4
mkdir -p $O
DRAW_ROWS=1 timeout -k 10 120 python -u scripts/draw_phases.py > $O/draw_phases_b1.txt 2>&1 &&
THR_ROWS=9 timeout -k 10 120 python -u scripts/thr_phases.py > $O/thr_phases_9.txt 2>&1 &&
(cd /tmp && export TMPDIR=/tmp CFG_NO_CPU=1 &&
 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_cfg1" -o run \
     -- python3 "$GRAFT_REPO_ROOT/scripts/config_timing.py" cfg1 > "$GRAFT_REPO_ROOT/$O/prof_cfg1.log" 2>&1)
echo "exit $?"
