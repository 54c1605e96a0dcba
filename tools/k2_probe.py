"""Stage times of one scheduling step (K2 refresh + keys-only eval) at config 3 for
binding logs of different node distributions: Zipf(1.1) (bench), uniform, and a
single node.  Uses the engine's stage timing (crane_dyn_set_profiling)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

dev = torch.device("cuda", 0)
spec = cd.default_policy_spec()
N, P, B = 100_000, 10_000, 1_000_000
c = synth.make_cluster(spec, N, P, n_bindings=B, seed=20250215 + 3000)
c.now, c.ds = synth.make_pods(P, seed=20250215 + 3)
rng = np.random.default_rng(1)
logs = {"zipf": c.b_node, "uniform": rng.integers(0, N, B).astype(np.int32), "one_node": np.full(B, 7, np.int32)}
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
d_now = torch.from_numpy(c.now).to(dev)
d_flags = torch.from_numpy(c.ds).to(dev)
d_keys = torch.empty(P, dtype=torch.int64, device=dev)
now = int(synth.NOW0_NS)
for name, bn in logs.items():
    eng = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    eng.upload_bindings(bn, c.b_ts)
    for _ in range(3):
        eng.refresh_hot_values_async(now, now, st.cuda_stream)
        eng.eval_keys_async(d_now, d_flags, d_keys, st.cuda_stream)
    st.synchronize()
    eng.set_profiling(True)
    acc = {}
    for _ in range(10):
        eng.refresh_hot_values_async(now, now, st.cuda_stream)
        eng.eval_keys_async(d_now, d_flags, d_keys, st.cuda_stream)
        for k, v in eng.stage_times():
            acc.setdefault(k, []).append(v)
    print(name, {k: round(float(np.median(v)) * 1e3, 1) for k, v in acc.items()}, "us", flush=True)
    eng.close()
