"""Print a rocprofv3 kernel_stats.csv compactly: calls, average / min / max µs, short name."""
import csv
import sys

for row in csv.DictReader(open(sys.argv[1])):
    name = row["Name"]
    short = name.split("(")[0] if name.startswith("void sd::") or name.startswith("sd::") else name[:60]
    print(f"{int(row['Calls']):6d} {float(row['AverageNs'])/1e3:8.2f} {float(row['MinNs'])/1e3:8.2f} "
          f"{float(row['MaxNs'])/1e3:8.2f}  {short}")
