"""Interleaved A/B of K3 variants / grid rounds in ONE process (guide §5.4 rule 24).

    python tools/k3_ab.py [--rounds 5] [--reps 5]
Prints per-(variant, rounds) median/min K3 time over config 3 and checks that
every variant returns identical keys.
"""
import argparse
import itertools
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="3,4")
ap.add_argument("--grid-rounds", default="8,16,32")
ap.add_argument("--pods", type=int, default=10_000)
ap.add_argument("--nodes", type=int, default=100_000)
args = ap.parse_args()

dev = torch.device("cuda", 0)
spec = cd.default_policy_spec()
c = synth.make_cluster(spec, args.nodes, args.pods, n_bindings=1_000_000, seed=20253215)
eng = cd.Engine(cd.Policy(spec), 0)
val, ts, _ = c.rows(eng.metric_names)
eng.upload_nodes(val, ts, c.hv, c.hv_ts)
eng.upload_bindings(c.b_node, c.b_ts)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
sh = st.cuda_stream
d_now = torch.from_numpy(c.now).to(dev)
d_flags = torch.from_numpy(c.ds).to(dev)
d_keys = torch.empty(args.pods, dtype=torch.int64, device=dev)
eng.refresh_hot_values_async(synth.NOW0_NS, synth.NOW0_NS, sh)
eng.node_pass_async(sh)
combos = list(itertools.product([int(v) for v in args.variants.split(",")], [int(r) for r in args.grid_rounds.split(",")]))
times = {cmb: [] for cmb in combos}
ref = None
for rnd in range(args.rounds):
    for v, gr in combos:
        os.environ["CRANE_K3_VARIANT"] = str(v)
        os.environ["CRANE_K3_ROUNDS"] = str(gr)
        eng.eval_keys_async(d_now, d_flags, d_keys, sh)  # warm this config
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            eng.eval_keys_async(d_now, d_flags, d_keys, sh)
            b.record(st)
            b.synchronize()
            times[(v, gr)].append(a.elapsed_time(b))
        k = d_keys.cpu().numpy()
        if ref is None:
            ref = k.copy()
        assert np.array_equal(k, ref), f"variant {v} rounds {gr} keys differ"
evals = args.pods * args.nodes
out = []
for (v, gr), t in times.items():
    med = float(np.median(t))
    out.append({"variant": v, "grid_rounds": gr, "median_ms": round(med, 4), "min_ms": round(float(np.min(t)), 4),
                "evals_per_s": round(evals / (med * 1e-3), 1)})
print(json.dumps(out, indent=1))
