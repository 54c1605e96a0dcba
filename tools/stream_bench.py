"""HBM roofline of the streaming kernels at large N, cold cache.

    python tools/stream_bench.py [--nodes 4000000] [--bindings 16000000] [--reps 5]

K1 (node pass) and K2 (hot-value counts) are timed separately with HIP events;
between reps a 1 GiB scratch buffer is written so the 256 MiB Infinity Cache
holds none of the inputs (MI355X_MICROARCH.md, Infinity Cache).
Algorithmic bytes:
  K1: 16*M (val+ts SoA) + 8*W (buckets read + zeroed) + sizeof(NodeRec) per node
  K2: 12 per binding (int32 node + int64 ts) + 4*W per node (bucket counts)
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
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--k1-threads", default="128,256")
ap.add_argument("--k2", default="binned,hash")
args = ap.parse_args()

dev = torch.device("cuda", 0)
spec = cd.default_policy_spec()
c = synth.make_cluster(spec, args.nodes, 1, n_bindings=args.bindings, seed=7)
eng = cd.Engine(cd.Policy(spec), 0)
val, ts, _ = c.rows(eng.metric_names)
eng.upload_nodes(val, ts, c.hv, c.hv_ts)
eng.upload_bindings(c.b_node, c.b_ts)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
sh = st.cuda_stream
scratch = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
M, W, N, B = len(eng.metric_names), len(spec["hotValue"]), args.nodes, args.bindings
REC = 160
k1_bytes = N * (16 * M + 8 * W + REC)
k2_bytes = B * 12 + 4 * W * N
t1, t2 = [], []
t1v = {v: [] for v in args.k1_threads.split(",")}
t2v = {v: [] for v in args.k2.split(",")}
for r in range(args.reps + 1):
    for v, k2 in zip(list(t1v) * len(t2v), sorted(list(t2v) * len(t1v))):
        os.environ["CRANE_K1_THREADS"] = v
        os.environ["CRANE_K2"] = k2
        scratch.fill_(r & 0xFF)
        a, b, d = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        a.record(st)
        eng.refresh_hot_values_async(synth.NOW0_NS, synth.NOW0_NS, sh)  # K2 (+ bucket memset on the first rep)
        b.record(st)
        scratch.fill_((r + 7) & 0xFF)
        c0 = torch.cuda.Event(enable_timing=True)
        c0.record(st)
        eng.node_pass_async(sh)  # K1
        d.record(st)
        d.synchronize()
        if r:  # rep 0 is warmup
            t2v[k2].append(a.elapsed_time(b))
            t1v[v].append(c0.elapsed_time(d))
best = min(t1v, key=lambda v: np.median(t1v[v]))
t1 = t1v[best]
best2 = min(t2v, key=lambda v: np.median(t2v[v]))
t2 = t2v[best2]
k1 = float(np.median(t1))
k2 = float(np.median(t2))
out = {"nodes": N, "bindings": B, "cold_cache": "1 GiB scratch write before each kernel",
       "k1_by_threads_ms": {v: round(float(np.median(x)), 4) for v, x in t1v.items()}, "k1_threads": best,
       "k2_by_mode_ms": {v: round(float(np.median(x)), 4) for v, x in t2v.items()}, "k2_mode": best2,
       "k1_node_pass": {"ms": round(k1, 4), "alg_bytes": k1_bytes, "GBps": round(k1_bytes / k1 / 1e6, 1),
                        "frac_of_8TBps": round(k1_bytes / k1 / 1e6 / 8000, 4)},
       "k2_hot_count": {"ms": round(k2, 4), "alg_bytes": k2_bytes, "GBps": round(k2_bytes / k2 / 1e6, 1),
                        "frac_of_8TBps": round(k2_bytes / k2 / 1e6 / 8000, 4)}}
print(json.dumps(out))
