"""Average rocprofv3 --pmc counter_collection CSVs per kernel.

    python tools/pmc_agg.py gpurun_out/pmc_<tag> [kernel-substring ...]
"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
pats = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    if pats and not any(p in k for p in pats):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:26s} {sum(v) / len(v):16.0f}  (n={len(v)})")
