set -eo pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py > gpurun_out/fused_tests.log 2>&1 || { tail -30 gpurun_out/fused_tests.log; exit 1; }
tail -2 gpurun_out/fused_tests.log
CONFIGS="new|;sl1|SPECDEC_LIB=libspecdec_sl1.so" REPS=3 bash scripts/gpu_ab_bench.sh
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase32.txt 2>&1
awk '/--- rep 3/,0' gpurun_out/phase32.txt | grep -A20 "fused verify roles"
