#!/bin/bash
# Copy a gpu_round.sh run's evidence from gpurun_out/ into profiles/ under a round tag.
# usage: scripts/save_round.sh r4a
set -e
TAG=$1
cd "$(dirname "$0")/.."
cp gpurun_out/prof/run_kernel_stats.csv profiles/${TAG}_kernel_stats_profile_only.csv
python scripts/trace_summary.py gpurun_out/prof profiles/${TAG}_kernel_trace_by_shape.csv > /dev/null
[ -f gpurun_out/prof.json ] && cp gpurun_out/prof.json profiles/${TAG}_prof_bench.json
[ -f gpurun_out/bench.json ] && cp gpurun_out/bench.json profiles/${TAG}_bench.json
[ -f gpurun_out/gpu_tests.log ] && tail -3 gpurun_out/gpu_tests.log > profiles/${TAG}_gpu_tests.txt
[ -f gpurun_out/ngs_timing.json ] && cp gpurun_out/ngs_timing.json profiles/${TAG}_ngram_store_timing.json
python scripts/pmc_summary.py gpurun_out ${TAG} engine_b32_g4_v128256 > /dev/null
python - "$TAG" <<'PY'
import csv, json, sys
tag = sys.argv[1]
b = json.load(open(f"profiles/{tag}_prof_bench.json"))
rows = list(csv.DictReader(open(f"profiles/{tag}_kernel_stats_profile_only.csv")))
k = b["roofline"]["kernel"]
for r in rows:
    if f"sd::{k}<" in r["Name"] or f"sd::{k}_lean<" in r["Name"]:
        print(f"{k}: bench {b['roofline']['kernel_ms']*1e6:.0f} ns/launch, rocprof avg {float(r['AverageNs']):.0f} ns "
              f"({r['Calls']} calls)")
print("profile-only run: value", b["value"], "ms/step", b["ms_per_step"], "frac", b["roofline"]["frac"])
PY
