#!/bin/bash
# GPU-box recipe: every GPU test, smoke(), one default bench line, the batch-1 A/B and a rocprofv3
# kernel summary of the bench.  Outputs under gpurun_out/.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/ > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 python scripts/b1_ab.py "" "LEAN_VERIFY=0" > gpurun_out/b1_ab.txt 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_bench.log 2>&1
