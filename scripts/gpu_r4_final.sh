set -eo pipefail
bash scripts/gpu_round.sh
tail -2 gpurun_out/gpu_tests.log
bash scripts/gpu_dp_rehearsal.sh
