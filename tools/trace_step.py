"""Per-workgroup phase timing of the step kernels (engine option "trace").

    python tools/trace_step.py [--config 3|4] [--reps 5]

Every workgroup of K2x (dedupe), K1 (+K3a) and K3s stamps s_memrealtime (100 MHz,
10 ns) at its phase boundaries; per kernel this prints the spread of workgroup
start times, each phase's duration (median / p90 / max over workgroups) and the
span first start -> last end, so the critical path of a launch can be read off.
With --queue the steps go to a dispatch queue (the headline's launch route); "timeline" gives the
launch-to-launch view of one step: each kernel's first workgroup start and last end relative to the
first kernel's start, and the gaps between the kernels.  --dt S moves the hot-value time by S
seconds per traced step (the delta form then adjusts its anchor by the bindings that changed).
Phases:
  K2 (delta form + K3p tiles): 0 start | 4 end
  K2x: 0 start | 1 bindings loaded + LDS cleared | 2 (node, bucket) aggregated | 3 counts/offsets written | 4 entries written
  K1 : 0 start | 1 SoA + K2 entries in (LDS counts) | 2 record computed | 3 step tables published | 4 stepped records emitted
  K3s: 0 start | 1 pods + producer counts in | 2 record rounds done | 3 uniform maxima reduced | 4 keys merged
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
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--opt", action="append", default=[], help="engine option name=value (repeatable)")
ap.add_argument("--nodes", type=int, default=0, help="override the config's node count")
ap.add_argument("--bindings", type=int, default=-1, help="override the config's binding count")
ap.add_argument("--queue", action="store_true", help="steps on a dispatch queue (crane_queue)")
ap.add_argument("--dt", type=int, default=0, help="hot-value time moved by this many seconds per traced step")
args = ap.parse_args()
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
spec = cd.default_policy_spec()
cfg = synth.CONFIGS[args.config]
N, P, B = cfg["nodes"], cfg["pods"], cfg["bindings"]
if args.config == 4:
    N //= 8
N = args.nodes or N
B = B if args.bindings < 0 else args.bindings
c = synth.make_cluster(spec, N, P, n_bindings=B, seed=20250215 + args.config * 1000)
c.now, c.ds = synth.make_pods(P, seed=20250215 + args.config)
eng = cd.Engine(cd.Policy(spec), 0)
for o in args.opt:
    k, v = o.split("=")
    eng.set_option(k, int(v))
val, ts, _ = c.rows(eng.metric_names)
eng.upload_nodes(val, ts, c.hv, c.hv_ts)
eng.upload_bindings(c.b_node, c.b_ts)
d_now = torch.from_numpy(c.now).to(dev)
d_flags = torch.from_numpy(c.ds).to(dev)
d_keys = torch.empty(P, dtype=torch.int64, device=dev)
now = int(synth.NOW0_NS)
q = cd.Queue(0) if args.queue else None
torch.cuda.synchronize()


def step(t):
    if q is not None:
        eng.step_keys_queue(t, t, d_now, d_flags, d_keys, q)
        q.wait()
    else:
        eng.step_keys_async(t, t, d_now, d_flags, d_keys, st.cuda_stream)
        st.synchronize()


for _ in range(3):
    step(now)
eng.set_option("trace", 1)
nwg = {0: -(-B // 2048), 1: -(-N // 256)}
res = {}
xcd = {}
acc = {k: [] for k in ("K2x", "K1", "K3s")}
import time  # noqa: E402
tl, host = [], []
for r in range(args.reps):
    h0 = time.perf_counter()
    step(now + (r + 1) * args.dt * 10**9)
    host.append((time.perf_counter() - h0) * 1e6)
    ends = {}
    for which, name in ((0, "K2x"), (1, "K1"), (2, "K3s")):
        t = eng.debug_trace(which, 65536).astype(np.int64)
        wg = np.nonzero(t[:, 0] > 0)[0]
        t = t[wg]
        acc[name].append(t)
        if len(t):
            ends[name] = (int(t[:, 0].min()), int(t[:, 4].max()))
    if len(ends) == 3:
        t0 = ends["K2x"][0]
        tl.append([(ends[k][i] - t0) / 100.0 for k in ("K2x", "K1", "K3s") for i in (0, 1)])
        # workgroup -> XCD placement: the XCD of each label (workgroup id % 8), as observed
        lab = {}
        for w, x in zip(wg % 8, t[:, 7]):
            lab.setdefault(int(w), set()).add(int(x))
        xcd.setdefault(name, []).append({k: sorted(v) for k, v in sorted(lab.items())})
    eng.set_option("trace", 1)  # clears the buffer for the next rep
out = {"config": args.config, "nodes": N, "pods": P, "bindings": B, "unit": "us"}
for name, runs in acc.items():
    if not all(len(t) for t in runs):
        continue  # (that kernel did not run: e.g. the binned K2 form at large N)
    spans, phases, starts, ends = [], {k: [] for k in range(4)}, [], []
    for t in runs:
        t0 = t[:, 0].min()
        spans.append((t[:, 4].max() - t0) / 100.0)
        starts.append((t[:, 0] - t0) / 100.0)
        ends.append((t[:, 4] - t0) / 100.0)
        for k in range(4):
            phases[k].append((t[:, k + 1] - t[:, k]) / 100.0)
    cat = lambda xs: np.concatenate(xs)  # noqa: E731
    q = lambda x: {"med": round(float(np.median(x)), 2), "p90": round(float(np.percentile(x, 90)), 2),  # noqa: E731
                   "max": round(float(np.max(x)), 2)}
    out[name] = {"workgroups": int(len(runs[0])), "span": round(float(np.median(spans)), 2),
                 "start": q(cat(starts)), "end": q(cat(ends)),
                 "phases": {f"{k}->{k + 1}": q(cat(phases[k])) for k in range(4)}}
    subs = {"K3s": {"0->5": (0, 5), "5->1": (5, 1), "1->6": (1, 6), "6->2": (6, 2)},  # pods in, records, pieces
            "K1": {"3->5": (3, 5), "5->6": (5, 6), "6->4": (6, 4)}}     # emitted, sorted, tile rows
    if name in subs:
        sub = subs[name]
        out[name]["sub"] = {k: q(cat([(t[:, b] - t[:, a]) / 100.0 for t in runs])) for k, (a, b) in sub.items()}
if tl:
    m = np.median(np.array(tl), axis=0)
    out["timeline"] = {"K2_end": round(m[1], 2), "K1_start": round(m[2], 2), "K1_end": round(m[3], 2),
                       "K3s_start": round(m[4], 2), "K3s_end": round(m[5], 2),
                       "gap_K2_K1": round(m[2] - m[1], 2), "gap_K1_K3s": round(m[4] - m[3], 2)}
out["host_step_us"] = round(float(np.median(host)), 2)  # enqueue -> completion seen, traced
out["xcd_of_label"] = {k: v[:3] for k, v in xcd.items()}
print(json.dumps(out))
