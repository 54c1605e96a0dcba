"""The drop-in plugin leg of bench.py alone (config-3 snapshot: 100k nodes by default), with the
same-harness CPU plugin on 4 pods, churn x1 / x10 / frozen, every pod checked by replay.
    python tools/dropin_probe.py [n_nodes] [n_pods]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]

import bench  # noqa: E402
import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
P = int(sys.argv[2]) if len(sys.argv) > 2 else 256
spec = cd.default_policy_spec()
c = synth.make_cluster(spec, N, P, seed=20253215)
c.now, c.ds = synth.make_pods(P, seed=20250218)
print(json.dumps(bench.dropin_leg(cd, spec, c, c.annotations(), c.now, c.ds, 16, 0, cpu_pods=4)), flush=True)
