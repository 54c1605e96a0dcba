"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (per dispatch),
plus the HBM traffic per launch corrected as MI355X_MICROARCH.md prescribes:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the
bytes of wide coalesced reads, so traffic_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

    python tools/pmc_summary.py <rocprofv3 output dir> [--config C]

With --config, the output is {"config", "src_hash", "kernels": {...}} (bench.py's
profiles/pmc/config<C>_<src_hash>.json format); the hash is bench.src_hash() of
this tree, i.e. of the kernels that were profiled.
"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
cfg = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--config" else None
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "End_Timestamp" in r:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
out = {}
for k, cs in acc.items():
    out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    if dur[k]:
        out[k]["_dispatch_ns"] = sum(dur[k]) / len(dur[k])
    if "FETCH_SIZE" in out[k] and "WRITE_SIZE" in out[k]:
        out[k]["traffic_bytes"] = (2 * out[k]["FETCH_SIZE"] + out[k]["WRITE_SIZE"]) * 1024
if cfg is not None:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # noqa: E402
    out = {"config": cfg, "src_hash": bench.src_hash(), "kernels": out}
print(json.dumps(out, indent=1, sort_keys=True))
