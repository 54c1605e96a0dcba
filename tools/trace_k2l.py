"""Phase stamps of the large-form K2 partition (k2l_partition) at the cold-leg size: per
region, the span of its hash phase (0->1), bin scan + count/offset words (1->2) and entry
writes + slot clears (2->3), and the gap since the same workgroup's previous region.

    python tools/trace_k2l.py [--opt name=value ...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--opt", action="append", default=[])
args = ap.parse_args()
spec = cd.default_policy_spec()
N, B = 4_000_000, 16_000_000
c = synth.make_cluster(spec, N, 8, n_bindings=B, seed=7)
eng = cd.Engine(cd.Policy(spec), 0)
for o in args.opt:
    k, v = o.split("=")
    eng.set_option(k, int(v))
eng.set_option("trace", 1)
val, ts, _ = c.rows(eng.metric_names)
eng.upload_nodes(val, ts, c.hv, c.hv_ts)
eng.upload_bindings(c.b_node, c.b_ts)
now = int(synth.NOW0_NS)
for _ in range(3):
    eng.refresh_hot_values(now, now)
nreg = -(-B // 4096) if "k2l_region=2048" not in args.opt else -(-B // 2048)
tr = eng.debug_trace(0, nreg).astype(np.int64)
us = lambda a: np.percentile(a, [50, 90, 99]).round(3).tolist()  # noqa: E731
live = (tr[:, :4] != 0).all(1)
in_win = np.array([(c.b_ts[r * (B // nreg):(r + 1) * (B // nreg)] > synth.NOW0 - 300).any() for r in range(nreg)])
out = {"regions": nreg, "stamped": int(live.sum()), "stamped_in_window": int((live & in_win).sum()),
       "in_window": int(in_win.sum())}
tr = tr[live]
t0 = tr[:, 0].min()
out["span_us"] = round((tr[:, 3].max() - t0) / 100.0, 2)
out["start_us"] = us((tr[:, 0] - t0) / 100.0)
for a, b in ((0, 1), (1, 2), (2, 3), (0, 3)):
    out[f"{a}->{b}"] = us((tr[:, b] - tr[:, a]) / 100.0)
ny = (N + 16383) // 16384
ty = eng.debug_trace(0, ny).astype(np.int64)[:, 4:7]
y0 = ty[:, 0].min()
out["y"] = {"bins": ny, "span_us": round((ty[:, 2].max() - y0) / 100.0, 2), "start_us": us((ty[:, 0] - y0) / 100.0),
            "gather": us((ty[:, 1] - ty[:, 0]) / 100.0), "flush": us((ty[:, 2] - ty[:, 1]) / 100.0)}
print(json.dumps(out))
