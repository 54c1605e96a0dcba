"""Writes the drop-in harness's input files (policy, config-3 snapshot, 256 pods) for running
tools/dropin_bench.cpp by hand, with no GPU work in this process.
    python tools/dropin_files.py <dir>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "crane-scheduler_amd")]

import bench  # noqa: E402
import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402

d = sys.argv[1]
os.makedirs(d, exist_ok=True)
spec = cd.default_policy_spec()
cfg = synth.CONFIGS[3]
c = synth.make_cluster(spec, cfg["nodes"], cfg["pods"], n_bindings=cfg["bindings"], seed=20250215 + 3000)
c.now, c.ds = synth.make_pods(cfg["pods"], seed=20250215 + 3)
print(bench._dropin_files(d, spec, c.annotations(), c.now[:256], c.ds[:256]))
