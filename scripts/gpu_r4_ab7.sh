set -eo pipefail
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
CONFIGS="new|;prev|SPECDEC_LIB=libspecdec_prev.so" REPS=3 bash scripts/gpu_ab_bench.sh
