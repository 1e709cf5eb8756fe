#!/bin/bash
# Round-5 configs[4] kernel trace on the current library (GPU box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b14
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp CFG_NO_CPU=1 &&
 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_cfg" -o run \
     -- python3 "$GRAFT_REPO_ROOT/scripts/config_timing.py" cfg4 > "$GRAFT_REPO_ROOT/$O/prof_cfg.log" 2>&1)
echo "exit $?"
