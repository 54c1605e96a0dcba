"""Per-block phases of the prefetching count pass (k1_count_pf, engine option k1_count_form 4)
at 4M nodes: each workgroup walks its blocks; per block it stamps 0 (its DMA landed, after the
barrier), 1 (values read, next DMA issued), 2 (record computed), 3 (slots exchanged, published).
The gap from a block's stamp 3 to the workgroup's next block's stamp 0 is the wait for the
next block's rows.

    python tools/trace_pf.py [--nodes 4000000] [--bindings 16000000] [--opt name=value ...]
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
ap.add_argument("--nodes", type=int, default=4_000_000)
ap.add_argument("--bindings", type=int, default=16_000_000)
ap.add_argument("--pods", type=int, default=10_000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--opt", action="append", default=[])
args = ap.parse_args()
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
spec = cd.default_policy_spec()
N, P, B = args.nodes, args.pods, args.bindings
c = synth.make_cluster(spec, N, P, n_bindings=B, seed=7)
eng = cd.Engine(cd.Policy(spec), 0)
for o in ["k1_split=1", "emit_threads=64", "k1_count_form=4"] + args.opt:
    k, v = o.split("=")
    eng.set_option(k, int(v))
val, ts, _ = c.rows(eng.metric_names)
eng.upload_nodes(val, ts, c.hv, c.hv_ts)
eng.upload_bindings(c.b_node, c.b_ts)
d_now = torch.from_numpy(c.now).to(dev)
d_flags = torch.from_numpy(c.ds).to(dev)
d_keys = torch.empty(P, dtype=torch.int64, device=dev)
now = int(synth.NOW0_NS)
for _ in range(3):
    eng.step_keys_async(now, now, d_now, d_flags, d_keys, st.cuda_stream)
nb = -(-N // 256)
q = lambda x: {"med": round(float(np.median(x)), 3), "p10": round(float(np.percentile(x, 10)), 3),  # noqa: E731
               "p90": round(float(np.percentile(x, 90)), 3)}
out = {"nodes": N, "bindings": B, "unit": "us", "runs": []}
for r in range(args.reps):
    eng.set_option("trace", 1)
    eng.step_keys_async(now, now, d_now, d_flags, d_keys, st.cuda_stream)
    st.synchronize()
    t = eng.debug_trace(1, nb).astype(np.int64)
    ok = t[:, 0] > 0
    t, wg = t[ok], t[ok, 6]
    t0 = t[:, 0].min()
    ph = {f"{k}->{k + 1}": q((t[:, k + 1] - t[:, k]) / 100.0) for k in range(3)}
    waits, per_wg = [], []
    for w in np.unique(wg):
        rows = t[wg == w]
        rows = rows[np.argsort(rows[:, 0])]
        waits.append((rows[1:, 0] - rows[:-1, 3]) / 100.0)
        per_wg.append(len(rows))
    waits = np.concatenate(waits) if waits else np.zeros(1)
    out["runs"].append({"span": round(float((t[:, 3].max() - t0) / 100.0), 2), "workgroups": int(len(np.unique(wg))),
                        "blocks_per_wg": q(np.array(per_wg)), "phases": ph, "wait_next_block": q(waits),
                        "first_block_start": q((t[:, 0] - t0)[np.isin(np.arange(len(t)), np.unique(wg, return_index=True)[1])] / 100.0)})
print(json.dumps(out))
