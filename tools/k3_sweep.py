"""Time the keys-only K3 launch (eval_keys_async) at BASELINE config 3 under
several environment settings, e.g. step-path grid sizes or K3 variants.

    python tools/k3_sweep.py CRANE_K3S_BLOCKS=1024,2048,4096 CRANE_K3_VARIANT=4,5
Each NAME=v1,v2 argument is swept on its own (others at their defaults).
Checks that every setting yields the same keys.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

REPS = 20
dev = torch.device("cuda", 0)
spec = cd.default_policy_spec()
cfg = synth.CONFIGS[3]
c = synth.make_cluster(spec, cfg["nodes"], cfg["pods"], n_bindings=cfg["bindings"], seed=20250215 + 3000)
c.now, c.ds = synth.make_pods(cfg["pods"], seed=20250215 + 3)
eng = cd.Engine(cd.Policy(spec), 0)
val, ts, _ = c.rows(eng.metric_names)
eng.upload_nodes(val, ts, c.hv, c.hv_ts)
eng.upload_bindings(c.b_node, c.b_ts)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
sh = st.cuda_stream
d_now = torch.from_numpy(c.now).to(dev)
d_flags = torch.from_numpy(c.ds).to(dev)
d_keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
eng.refresh_hot_values_async(synth.NOW0_NS, synth.NOW0_NS, sh)
eng.node_pass_async(sh)


def timed():
    for _ in range(3):
        eng.eval_keys_async(d_now, d_flags, d_keys, sh)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(REPS)]
    for a, b in ev:
        a.record(st)
        eng.eval_keys_async(d_now, d_flags, d_keys, sh)
        b.record(st)
    st.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3, d_keys.cpu().numpy().copy()


out = {}
base_us, ref = timed()
out["default"] = round(base_us, 2)
for arg in sys.argv[1:]:
    name, vals = arg.split("=", 1)
    old = os.environ.get(name)
    for v in vals.split(","):
        os.environ[name] = v
        us, k = timed()
        out[f"{name}={v}"] = round(us, 2)
        if not np.array_equal(k, ref):
            out[f"{name}={v}_MISMATCH"] = int((k != ref).sum())
    if old is None:
        del os.environ[name]
    else:
        os.environ[name] = old
print(json.dumps({"us_per_eval_keys_launch": out, "pods": cfg["pods"], "nodes": cfg["nodes"]}))
