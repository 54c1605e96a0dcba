"""The drop-in plugin leg of bench.py alone (config-3 snapshot: 100k nodes, 64 pods), with the
same-harness CPU plugin on 4 pods.   python tools/dropin_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]

import bench  # noqa: E402
import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

spec = cd.default_policy_spec()
c = synth.make_cluster(spec, 100_000, 10_000, seed=20253215)
c.now, c.ds = synth.make_pods(10_000, seed=20250218)
e = cd.Engine(cd.Policy(spec), 0)
val, ts, _ = c.rows(e.metric_names)
e.upload_nodes(val, ts, c.hv, c.hv_ts)
_, _, ref_ch, _ = e.eval(c.now[:64], c.ds[:64])
e.close()
print(json.dumps(bench.dropin_leg(cd, spec, c.annotations(), c.now[:64], c.ds[:64], ref_ch, 16, cpu_pods=4)))
