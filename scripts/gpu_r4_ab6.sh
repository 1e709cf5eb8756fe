set -eo pipefail
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -8 gpurun_out/gpu_tests.log
CONFIGS="new|;prev|SPECDEC_LIB=libspecdec_prev.so" REPS=3 bash scripts/gpu_ab_bench.sh
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase32.txt 2>&1
awk '/--- rep 3/,0' gpurun_out/phase32.txt | grep -A40 "fused verify roles"
