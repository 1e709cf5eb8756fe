set -eo pipefail
timeout -k 10 200 python scripts/phase_timing.py > gpurun_out/phase32.txt 2>&1
grep -A20 "fused verify roles" gpurun_out/phase32.txt | tail -21
