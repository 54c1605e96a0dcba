"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (per dispatch)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
out = {}
for k, cs in acc.items():
    out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    out[k]["_dispatch_ns"] = sum(dur[k]) / len(dur[k])
print(json.dumps(out, indent=1))
