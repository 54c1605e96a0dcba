"""Print a rocprofv3 kernel_stats.csv as `calls  avg_us  pct  kernel` lines.

    python tools/kstats.py gpurun_out/<tag>/prof/bench_kernel_stats.csv
"""
import csv
import re
import sys

for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*\)$", "", r["Name"]).replace("void ", "")
        print(f"{int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:10.2f} us {float(r['Percentage']):6.2f}%  {name}")
