"""Repeat test_greedy_then_eval_consistent's sequence (greedy, re-upload nodes, eval) with
variants, counting chosen-node mismatches against the oracle: after greedy (step path,
matrix path via keys_path=1), eval without greedy, and with freed device memory filled
with a pattern before each engine (uninitialised-scratch probe).   Diagnostic only."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "crane-scheduler_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402
import crane_dyn as cd  # noqa: E402
from crane_dyn import synth  # noqa: E402
from helpers import engine_for, oracle_soa  # noqa: E402


def run(variant, form, seed, fill):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 500, 50, n_bindings=3000, seed=seed)
    if fill is not None:
        t = torch.full((64 << 20,), fill, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        del t
        torch.cuda.empty_cache()
    opts = {"greedy_form": form}
    if variant == "matrix":
        opts["keys_path"] = 1
    eng = engine_for(spec, c, opts=opts)
    eng.upload_bindings(c.b_node, c.b_ts)
    if variant != "nogreedy":
        eng.greedy(50, int(c.now[0]), c.ds)
    eng.upload_nodes(*c.rows(eng.metric_names)[:2], c.hv, c.hv_ts)
    _, _, ch, _ = eng.eval(c.now, c.ds)
    _, _, ch2, _ = eng.eval(c.now, c.ds)
    want = oracle_soa(spec, c, want_matrix=False)[2]
    return int((ch != want).sum()), int((ch2 != want).sum()), int(ch[0]), int(want[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    out = {}
    for fill in (None, 0xFF, 0x00, 0x5A):
        for variant in ("greedy", "matrix", "nogreedy"):
            for form in (0, 1):
                bad, bad2, ex = 0, 0, []
                for r in range(a.reps):
                    seed = 8 + (r % 4)
                    m1, m2, g, w = run(variant, form, seed, fill)
                    bad += m1 > 0
                    bad2 += m2 > 0
                    if (m1 or m2) and len(ex) < 3:
                        ex.append((seed, m1, m2, g, w))
                k = f"fill={fill} {variant} form={form}"
                out[k] = {"runs": a.reps, "first_eval_bad": bad, "second_eval_bad": bad2, "examples": ex}
                print(k, out[k], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
