set -eo pipefail
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for r in 1 2; do
  timeout -k 10 300 python scripts/b1_ab.py "" > gpurun_out/b1_new_$r.txt 2>&1
  SPECDEC_LIB=libspecdec_prev.so timeout -k 10 300 python scripts/b1_ab.py "" > gpurun_out/b1_prev_$r.txt 2>&1
done
tail -n1 gpurun_out/b1_new_*.txt gpurun_out/b1_prev_*.txt
