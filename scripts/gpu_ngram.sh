#!/bin/bash
# GPU-box recipe: device n-gram store tests (store + drop-in loop goldens), then its timing.
set -eo pipefail
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_ngram_store.py tests/test_gpu_parity.py -k ngram > gpurun_out/ngs_tests.log 2>&1
timeout -k 10 200 python scripts/ngram_store_timing.py > gpurun_out/ngs_timing.json 2> gpurun_out/ngs_timing.err
