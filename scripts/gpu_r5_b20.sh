#!/bin/bash
# Round-5 STREAM engine step kernel trace on the current library (GPU box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b20
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp &&
 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_stream" -o run \
     -- python3 "$GRAFT_REPO_ROOT/scripts/stream_ab.py" > "$GRAFT_REPO_ROOT/$O/prof_stream.log" 2>&1)
echo "exit $?"
