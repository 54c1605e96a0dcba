"""HBM roofline of the streaming kernels of one scheduling step at large N, cold cache.

    python tools/stream_bench.py [--nodes 4000000] [--bindings 16000000] [--pods 10000] [--reps 5]

One step = K2 refresh (the binned form at this size, or the hash form) then a
keys-only eval (k3p_pods, k1_node_pass+k3a_steps or its split form k1_node_pass+k3a_count +
k3a_emit, k3s_eval).  Kernel times come
from the engine's dispatch-stamped events (crane_dyn_set_profiling).  Before
the refresh and before the eval a 1 GiB scratch buffer is written (--flush write:
the Infinity Cache is then full of dirty lines that are written back while the
timed kernels read) or read (--flush read: clean lines), so the 256 MiB Infinity
Cache holds none of the inputs (MI355X_MICROARCH.md).
Algorithmic bytes:
  k2 (all K2 kernels)     : 12 per binding read + 4*W per node (window counts written)
  k1_node_pass+k3a_steps  : 16*M (val+ts SoA) + 8*W (buckets read + zeroed) + 8 (hot value) per node
                            (+ sizeof(NodeRec) with --keep-records: the keys-only pass keeps them in LDS)
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
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--k2", default="auto,hash")
ap.add_argument("--keep-records", action="store_true")
ap.add_argument("--flush", default="read", choices=("write", "read"),
                help="evict the caches by writing the 1 GiB scratch (its dirty lines are written back during "
                     "the timed kernels) or by reading it (clean lines)")
ap.add_argument("--opt", action="append", default=[], help="engine option name=value (repeatable)")
args = ap.parse_args()

dev = torch.device("cuda", 0)
spec = cd.default_policy_spec()
N, B, P = args.nodes, args.bindings, args.pods
c = synth.make_cluster(spec, N, P, n_bindings=B, seed=7)
c.now, c.ds = synth.make_pods(P, seed=8)
eng = cd.Engine(cd.Policy(spec), 0)
eng.set_option("k1_keep_records", int(args.keep_records))
for o in args.opt:
    k, v = o.split("=")
    eng.set_option(k, int(v))
val, ts, _ = c.rows(eng.metric_names)
eng.upload_nodes(val, ts, c.hv, c.hv_ts)
eng.upload_bindings(c.b_node, c.b_ts)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
sh = st.cuda_stream
d_now = torch.from_numpy(c.now).to(dev)
d_flags = torch.from_numpy(c.ds).to(dev)
d_keys = torch.empty(P, dtype=torch.int64, device=dev)
scratch = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
M, W = len(eng.metric_names), len(spec["hotValue"])
REC = 160  # sizeof(NodeRec<4, 6>)
now = int(synth.NOW0_NS)
max_tr = max(tr for tr, _ in spec["hotValue"]) // 10**9
b_in = int((c.b_ts > now // 10**9 - max_tr).sum())
alg = {
    "k2 (all K2 kernels)": B * 12 + 4 * W * N,
    "k1_node_pass+k3a_steps": N * (16 * M + 8 * W + 8 + (REC if args.keep_records else 0)),
    "k1_node_pass+k3a_count": N * (16 * M + 8 * W + 8),  # split form (k3a_emit builds the tables after it)
    "k1 split total (count + emit)": N * (16 * M + 8 * W + 8),
}
sink = torch.empty(1, dtype=torch.int64, device=dev)


def flush(r):
    if args.flush == "write":
        scratch.fill_(r & 0xFF)
    else:
        torch.sum(scratch.view(torch.int64), dim=0, keepdim=True, out=sink)


res = {}
keys_ref = None
for k2 in args.k2.split(","):
    eng.set_option("k2_form", {"auto": 0, "binned": 1, "hash": 2}[k2])
    acc = {}
    for r in range(args.reps + 1):
        flush(r)
        eng.set_profiling(True)
        eng.refresh_hot_values_async(now, now, sh)
        t_k2 = eng.stage_times()
        flush(r + 7)
        eng.set_profiling(True)
        eng.eval_keys_async(d_now, d_flags, d_keys, sh)
        t_ev = eng.stage_times()
        if r:  # rep 0 is warmup
            for name, t in t_k2 + t_ev:
                acc.setdefault(name, []).append(t)
            acc.setdefault("k2 (all K2 kernels)", []).append(sum(t for _, t in t_k2))
            split = [t for name, t in t_ev if name in ("k1_node_pass+k3a_count", "k3a_emit")]
            if len(split) == 2:  # the split form's two kernels together build what the fused one does
                acc.setdefault("k1 split total (count + emit)", []).append(sum(split))
    eng.set_profiling(False)
    keys = d_keys.cpu().numpy()
    if keys_ref is None:
        keys_ref = keys
    assert np.array_equal(keys, keys_ref), f"K2 mode {k2} changed the choices"
    stages = {}
    for name, v in acc.items():
        ms = float(np.median(v))
        e = {"ms": round(ms, 4)}
        if name in alg:
            gbs = alg[name] / (ms * 1e-3) / 1e9
            e.update({"alg_bytes": alg[name], "GBps": round(gbs, 1), "frac_of_8TBps": round(gbs / 8000, 4)})
        stages[name] = e
    res[k2] = stages
out = {"keep_records": args.keep_records, "nodes": N, "bindings": B, "bindings_in_window": b_in, "pods": P,
       "cold_cache": f"1 GiB scratch {args.flush} before the refresh and before the eval", "by_k2_mode": res}
print(json.dumps(out))
