"""K3m launch-geometry sweep: nodes per lane (matrix_vec) x pods per workgroup
(matrix_chunk) on the config-2 and config-3 shapes; kernel times are the
dispatch-stamped durations; every geometry's matrices and keys must equal the
automatic geometry's bit for bit.

    python tools/matrix_probe.py [--reps 10]
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
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--configs", default="2,3")
args = ap.parse_args()
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
spec = cd.default_policy_spec()
res = {}
for cid in [int(x) for x in args.configs.split(",")]:
    N, P = synth.CONFIGS[cid]["nodes"], synth.CONFIGS[cid]["pods"]
    c = synth.make_cluster(spec, N, P, seed=20250215 + cid)
    eng = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    ff = torch.empty((P, N), dtype=torch.int8, device=dev)
    sc = torch.empty((P, N), dtype=torch.int8, device=dev)
    keys = torch.empty(P, dtype=torch.int64, device=dev)
    ref = None
    out = {}
    combos = [(v, c) for v in (0, 1, 4, 8, 16) for c in (0, 16, 64, 256, 1024)]
    for vec, chunk in combos:
        if True:
            eng.set_option("matrix_vec", vec)
            eng.set_option("matrix_chunk", chunk)
            ff.fill_(99)
            sc.fill_(99)
            eng.eval_matrix_async(d_now, d_flags, ff, sc, keys, stream=st.cuda_stream)
            st.synchronize()
            cur = (ff.clone(), sc.clone(), keys.clone())
            if ref is None:
                ref = cur
            same = all(torch.equal(a, b) for a, b in zip(cur, ref))
            eng.set_profiling(True)
            ts_ = []
            for _ in range(args.reps):
                eng.eval_matrix_async(d_now, d_flags, ff, sc, keys, stream=st.cuda_stream)
                ts_ += [t for n, t in eng.stage_times() if n.startswith("k3m")]
            eng.set_profiling(False)
            ms = float(np.median(ts_))
            out[f"vec{vec}_chunk{chunk}"] = {"ms": round(ms, 4), "same": same,
                                             "GBps_written": round(2 * P * N / (ms * 1e-3) / 1e9, 1)}
    # the same automatic geometry without keys / without first-fail, and a plain fill of both matrices
    eng.set_option("matrix_vec", 0)
    eng.set_option("matrix_chunk", 0)
    for label, kk, f in (("auto_nokeys", None, ff), ("auto_score_only", keys, None)):
        eng.set_profiling(True)
        ts_ = []
        for _ in range(args.reps):
            eng.eval_matrix_async(d_now, d_flags, f, sc, kk, stream=st.cuda_stream)
            ts_ += [t for n, t in eng.stage_times() if n.startswith("k3m")]
        eng.set_profiling(False)
        out[label] = {"ms": round(float(np.median(ts_)), 4)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.reps):
        ff.fill_(1)
        sc.fill_(2)
    e1.record(st)
    st.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    out["torch_fill_both"] = {"ms": round(ms, 4), "GBps_written": round(2 * P * N / (ms * 1e-3) / 1e9, 1)}
    res[f"config{cid}"] = out
    eng.close()
    del ff, sc
print(json.dumps(res))
