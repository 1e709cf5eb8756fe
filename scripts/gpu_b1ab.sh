#!/bin/bash
# GPU-box recipe: batch-1 work — verify tests, configs[1] step times (A/B arguments in $AB; a second
# library build in $LIB2 for a compile-time A/B), and the phase stamps of configs[1]'s multinomial
# verify.  Outputs under gpurun_out/.
set -eo pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_lean_verify.py tests/test_gpu_parity.py tests/test_gpu_perfmode.py tests/test_gpu_greedy.py tests/test_gpu_engine_surface.py tests/test_gpu_errors.py tests/test_gpu_threshold.py > gpurun_out/b1_tests.log 2>&1
timeout -k 10 300 python scripts/b1_ab.py "" $AB > gpurun_out/b1_ab.txt 2>&1
if [ -n "$LIB2" ]; then
  SPECDEC_LIB=$LIB2 timeout -k 10 300 python scripts/b1_ab.py "" $AB > gpurun_out/b1_ab_lib2.txt 2>&1
fi
B=1 RULE=spec timeout -k 10 120 python scripts/phase_timing.py > gpurun_out/b1_verify_phases.txt 2>&1
