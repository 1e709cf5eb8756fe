#!/bin/bash
# Round-5 nucleus lean-verify phases (GPU box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b10
mkdir -p $O
PROC=nucleus B=1 RULE=spec timeout -k 10 120 python -u scripts/phase_timing.py > $O/lean_nuc_phases.txt 2>&1 &&
B=1 RULE=spec timeout -k 10 120 python -u scripts/phase_timing.py > $O/lean_phases.txt 2>&1
echo "exit $?"
