set -eo pipefail
SKIP_TESTS=1 SKIP_NGS=1 bash scripts/gpu_round.sh
CONFIGS="base|;pipe8|SPECDEC_LIB=libspecdec_pipe8.so;pipe8_st8|SPECDEC_LIB=libspecdec_pipe8.so SD_STATS_STAGES=8;st8|SD_STATS_STAGES=8;dec|SD_DEC_IN_SAMPLE=1" REPS=2 bash scripts/gpu_ab_bench.sh
