"""Timing of framework-level selection (bench.select_leg) at the config-3 shape.

    python tools/select_probe.py [option=value ...]   (engine options, e.g. sel_chain=1)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

spec = cd.default_policy_spec()
c = synth.make_cluster(spec, 100000, 10000, seed=7)
e = cd.Engine(cd.Policy(spec), 0)
names = e.metric_names
e.close()
val, ts, _ = c.rows(names)
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
torch.cuda.set_stream(st)
print(json.dumps(bench.select_leg(cd, spec, dev, st, val, ts, c.hv, c.hv_ts, c.now, c.ds, opts=sys.argv[1:])))
