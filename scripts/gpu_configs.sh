#!/bin/bash
# GPU-box recipe: every GPU test, then the per-config step timing (scripts/config_timing.py) and one
# bench line on HEAD.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 400 python scripts/config_timing.py ${CFG:-cfg1 cfg4 sweep} > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err
