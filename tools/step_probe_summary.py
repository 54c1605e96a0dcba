"""Summary of tools/step_probe.sh output: per kernel span and median phases, bench stage times."""
import json
import sys

d0 = sys.argv[1]
for f in ("trace3.json", "trace4.json"):
    d = json.load(open(f"{d0}/{f}"))
    for k in ("K2x", "K1", "K3s"):
        print(f, k, d[k]["workgroups"], d[k]["span"], {p: v["med"] for p, v in d[k]["phases"].items()},
              "p90end", d[k]["end"]["p90"], {p: v["med"] for p, v in d[k].get("sub", {}).items()})
for f in ("b3.log", "b4.log"):
    d = json.loads(open(f"{d0}/{f}").read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d.get("kernel_ms"))
