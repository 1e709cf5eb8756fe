#!/bin/bash
# GPU-box recipe: per-workgroup phase timing of the bench's draw and verify kernels
set -eo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/draw_timing.py > gpurun_out/draw_phase.log 2>&1
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase.log 2>&1
