"""Throughput of the keys-only step with K independent pod batches in flight: K engines
(each its own node SoA, binding log and scratch) on K HIP streams, batch i on engine i % K.
Every batch does the whole step (K2x+K3p, K1+K3a, K3s); the streams let one batch's
latency-bound kernels overlap another's.  Keys of every engine are checked equal.

    python tools/inflight_probe.py [--config 3] [--steps 200] [--inflight 1,2,3,4]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]

import torch  # noqa: E402

import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--inflight", default="1,2,3,4")
ap.add_argument("--bound", action="store_true", help="pre-bound step functions (Engine.step_keys_fn)")
ap.add_argument("--threads", action="store_true", help="one host thread per engine enqueues its batches")
ap.add_argument("--opt", action="append", default=[], help="engine option name=value (repeatable)")
ap.add_argument("--start-at", type=float, default=0.0,
                help="time.time() at which the timed loop starts (several processes on one GPU timed together)")
args = ap.parse_args()
dev = torch.device("cuda", 0)
spec = cd.default_policy_spec()
cfg = synth.CONFIGS[args.config]
N, P, B = cfg["nodes"], cfg["pods"], cfg["bindings"]
if args.config == 4:
    N //= 8
c = synth.make_cluster(spec, N, P, n_bindings=B, seed=20250215 + args.config * 1000)
c.now, c.ds = synth.make_pods(P, seed=20250215 + args.config)
now = int(synth.NOW0_NS)
out = {"bound": args.bound, "threads": args.threads, "config": args.config, "nodes": N, "pods": P, "bindings": B, "opts": args.opt}
for K in [int(x) for x in args.inflight.split(",")]:
    engs, streams, keys = [], [], []
    for _ in range(K):
        e = cd.Engine(cd.Policy(spec), 0)
        for o in args.opt:
            k_, v_ = o.split("=")
            e.set_option(k_, int(v_))
        val, ts, _ = c.rows(e.metric_names)
        e.upload_nodes(val, ts, c.hv, c.hv_ts)
        e.upload_bindings(c.b_node, c.b_ts)
        engs.append(e)
        streams.append(torch.cuda.Stream(dev))
        keys.append(torch.empty(P, dtype=torch.int64, device=dev))
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)

    fns = [e.step_keys_fn(d_now, d_flags, keys[j], streams[j].cuda_stream) for j, e in enumerate(engs)]

    def step(i):
        j = i % K
        if args.bound:
            fns[j](now, now)
        else:
            engs[j].step_keys_async(now, now, d_now, d_flags, keys[j], streams[j].cuda_stream)

    for i in range(10):
        step(i)
    torch.cuda.synchronize()
    if args.start_at:
        time.sleep(max(0.0, args.start_at - time.time()))
    t0 = time.perf_counter()
    w0 = time.time()
    if args.threads:
        def run(j):
            f = fns[j]
            for _ in range(j, args.steps, K):
                f(now, now)
        th = [threading.Thread(target=run, args=(j,)) for j in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    else:
        for i in range(args.steps):
            step(i)
    t_host = time.perf_counter() - t0  # enqueue time alone
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / args.steps
    same = all(torch.equal(keys[0], k) for k in keys)
    out[f"inflight{K}"] = {"ms_per_step": round(ms, 4), "host_enqueue_ms_per_step": round(t_host * 1e3 / args.steps, 4),
                           "keys_equal": same, "wall": [round(w0, 6), round(w0 + ms * args.steps / 1e3, 6)]}
    for e in engs:
        e.close()
print(json.dumps(out))
