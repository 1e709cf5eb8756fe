#!/bin/bash
# GPU-box A/B of k_draw_lean builds: the draw tests under the candidate library, then the draw
# launch time (bench shape and batch 1) and the configs[1] step, alternating libraries.
# usage: [TESTS=...] LIBS="libspecdec.so libspecdec_x.so" CAND=libspecdec_x.so bash scripts/gpu_ab_draw.sh
set -eo pipefail
R0=$GRAFT_REPO_ROOT
cd $R0
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
TESTS=${TESTS:-"tests/test_gpu_draw.py tests/test_gpu_perfmode.py tests/test_gpu_greedy.py tests/test_gpu_window.py tests/test_gpu_errors.py tests/test_gpu_engine_surface.py"}
SPECDEC_LIB=$CAND timeout -k 10 300 $T $TESTS > gpurun_out/ab_tests.log 2>&1
for rep in 1 2; do
  for L in $LIBS; do
    for R in 32 1; do
      SPECDEC_LIB=$L R=$R timeout -k 10 120 python scripts/draw_bench.py >> gpurun_out/ab_draw.txt 2>&1
    done
  done
done
for L in $LIBS; do
  echo "== $L" >> gpurun_out/ab_b1.txt
  SPECDEC_LIB=$L timeout -k 10 200 python scripts/b1_ab.py "" >> gpurun_out/ab_b1.txt 2>&1
done
