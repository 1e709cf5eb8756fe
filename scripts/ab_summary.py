"""Summarise gpurun_out/ab_* (scripts/gpu_ab_env.sh): ms/step, phases and per-kernel averages."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(out, "ab_*.json"))):
    name = os.path.basename(f)[3:-5]
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(name, "no bench line:", e)
        continue
    print(f"{name:16s} {j['ms_per_step']*1e3:7.2f} us/step  tok/s {j['value']/1e6:6.3f}M  acc {j['acceptance_rate']:.4f}  "
          f"draws {j['phases_ms']['draws']*1e3:6.2f} verify {j['phases_ms']['verify']*1e3:6.2f}  "
          f"k_stats(ev) {j['roofline']['kernel_ms']*1e3:6.2f}")
    ks = os.path.join(out, f"ab_prof_{name}", "run_kernel_stats.csv")
    if os.path.exists(ks):
        for row in csv.DictReader(open(ks)):
            if "sd::" in row["Name"]:
                print(f"    {int(row['Calls']):6d} {float(row['AverageNs'])/1e3:7.2f} us  {row['Name'][:70]}")
