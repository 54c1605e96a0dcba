"""Generate the committed golden fixtures (TEST INFRASTRUCTURE).

    python tests/golden/make_golden.py

Writes tests/golden/kats.json (hand-derived known-answer tests, SURVEY.md
§8c KAT-1..11 plus edge cases) and tests/golden/cluster_small.json (a seeded
64-node x 12-pod cluster with well-formed and malformed annotations).  The
expected outputs come from pyref.py, the independent pure-Python restatement
of /root/reference/pkg/plugins/dynamic/{plugins,stats}.go.  The KAT values the
survey derived by hand are asserted here before anything is written, so a
drift in pyref cannot silently rewrite them.

Parity is unpinned by the reference itself: it ships no tests or fixtures for
this path and its Go toolchain is absent.
"""
from __future__ import annotations

import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pyref  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
NOW0 = 1792065600  # 2026-10-15T20:00:00+08:00 (KAT-9)
NOW0_NS = NOW0 * 10**9
METRICS = [n for n, _ in pyref.default_policy()["syncPolicy"]]


def anno_of(usages, age_s=0, hv=None, hv_age_s=0):
    a = {}
    for name, u in zip(METRICS, usages):
        if u is None:
            continue
        a[name] = f"{u},{pyref.format_local(NOW0 - age_s)}" if not isinstance(u, tuple) else f"{u[0]},{pyref.format_local(NOW0 - u[1])}"
    if hv is not None:
        a[pyref.NODE_HOT_VALUE] = f"{hv},{pyref.format_local(NOW0 - hv_age_s)}"
    return a


def kat(name, anno, expect_filter, expect_score, now_ns=NOW0_NS, ds=False, policy=None, note=""):
    pol = policy or pyref.default_policy()
    f = pyref.filter_node(pol, anno, now_ns, ds)
    s = pyref.score_node(pol, anno, now_ns)
    assert f == expect_filter, (name, f, expect_filter)
    assert s == expect_score, (name, s, expect_score)
    return {"name": name, "note": note, "annotations": anno, "now_ns": now_ns, "daemonset": ds,
            "policy": policy_json(pol), "expect_filter": f, "expect_score": s}


def policy_json(pol):
    return {"syncPolicy": [[n, p] for n, p in pol["syncPolicy"]],
            "predicate": [[n, l] for n, l in pol["predicate"]],
            "priority": [[n, w] for n, w in pol["priority"]],
            "hotValue": [[t, c] for t, c in pol["hotValue"]]}


def make_kats():
    D = pyref.default_policy()
    ks = []
    # KAT-1: all usages 0.5 -> 50; hv=3 -> 20.  Filter: 0.5 < limits.
    ks.append(kat("KAT-1a", anno_of([0.5] * 6), -1, 50))
    ks.append(kat("KAT-1b", anno_of([0.5] * 6, hv=3), -1, 20))
    # KAT-2: [0.1..0.6] -> 62; metric 1 stale -> 53 (weight still 2.0)
    ks.append(kat("KAT-2a", anno_of([0.1, 0.2, 0.3, 0.4, 0.5, 0.6]), -1, 62))
    ks.append(kat("KAT-2b", anno_of([(0.1, 8 * 60 + 1), 0.2, 0.3, 0.4, 0.5, 0.6]), -1, 53,
                  note="cpu_usage_avg_5m written 8m01s ago: stale (3m+5m)"))
    # KAT-3: FMA trap: q = 48.99999999999999 -> 48 (FMA-contracted build gives 49)
    ks.append(kat("KAT-3", anno_of([0.21, 0.78, 0.34, 0.98, 0.61, 0.39]), 1, 48,
                  note="filter: cpu_usage_max_avg_1h 0.78 > 0.75"))
    # KAT-4: q = 31.0 exactly -> 31 (FMA gives 30.999999999999996 -> 30)
    ks.append(kat("KAT-4", anno_of([0.292, 0.424, 0.488, 0.987, 0.935, 0.945]), 2, 31))
    # KAT-5: all 1.5 -> q = -50 -> clamp 0; first predicate fails
    ks.append(kat("KAT-5", anno_of([1.5] * 6), 0, 0))
    # KAT-6: all 0 -> 100; hv=3 -> 70
    ks.append(kat("KAT-6a", anno_of([0.0] * 6), -1, 100))
    ks.append(kat("KAT-6b", anno_of([0.0] * 6, hv=3), -1, 70))
    # KAT-7: strict '>' and maxLimitPecent 0
    ks.append(kat("KAT-7a", anno_of([0.65, 0.1, 0.1, 0.1, 0.1, 0.1]), -1, 84))
    ks.append(kat("KAT-7b", anno_of([0.65001, 0.1, 0.1, 0.1, 0.1, 0.1]), 0, 84))
    P0 = dict(D)
    P0["predicate"] = [("cpu_usage_avg_5m", 0.0)] + D["predicate"][1:]
    ks.append(kat("KAT-7c", anno_of([0.99, 0.1, 0.1, 0.1, 0.1, 0.1]), -1, 81, policy=P0,
                  note="maxLimitPecent 0 disables the predicate"))
    # KAT-8: staleness boundaries.  period 3m -> 8m active.
    ks.append(kat("KAT-8a", anno_of([(0.9, 480), 0.1, 0.1, 0.1, 0.1, 0.1]), -1, 81,
                  note="ts = now-480s: now < ts+8m is false -> stale -> not overloaded"))
    ks.append(kat("KAT-8b", anno_of([(0.9, 479), 0.1, 0.1, 0.1, 0.1, 0.1]), 0, 82))
    ks.append(kat("KAT-8c", anno_of([0.0] * 6, hv=3, hv_age_s=300), -1, 100, note="hot value 5m window: stale"))
    ks.append(kat("KAT-8d", anno_of([0.0] * 6, hv=3, hv_age_s=299), -1, 70))
    # KAT-10: NaN usage passes validation; int(NaN) = INT64_MIN
    ks.append(kat("KAT-10a", anno_of(["NaN", 0.1, 0.1, 0.1, 0.1, 0.1]), -1, 0))
    ks.append(kat("KAT-10b", anno_of(["NaN", 0.1, 0.1, 0.1, 0.1, 0.1], hv=1), -1, 100,
                  note="INT64_MIN - 10 wraps to INT64_MAX-9 -> clamp 100"))
    # edge: malformed / missing / negative / Inf / range
    ks.append(kat("E-missing", anno_of([None, 0.1, 0.1, 0.1, 0.1, 0.1]), -1, 81))
    a = anno_of([0.9] * 6)
    a["cpu_usage_avg_5m"] = "0.9"  # no timestamp: Split gives 1 part
    a["cpu_usage_max_avg_1h"] = "0.9,2026-10-15T20:00:00Z,x"  # 3 parts
    a["mem_usage_avg_5m"] = "-0.5," + pyref.format_local(NOW0)  # negative
    a["mem_usage_max_avg_1h"] = " 0.9," + pyref.format_local(NOW0)  # leading space: syntax
    ks.append(kat("E-malformed", a, -1, 4, note="only the two *_1d metrics are usable: q = 4.999999999999999"))
    a = anno_of([0.1] * 6)
    a["cpu_usage_avg_5m"] = "+Inf," + pyref.format_local(NOW0)
    ks.append(kat("E-inf", a, 0, 0, note="+Inf > 0.65; score -Inf -> INT64_MIN -> 0"))
    a = anno_of([0.1] * 6)
    a["cpu_usage_avg_5m"] = "1e400," + pyref.format_local(NOW0)
    ks.append(kat("E-range", a, -1, 81, note="ParseFloat ErrRange -> error -> stale-like"))
    a = anno_of([0.1] * 6)
    a["cpu_usage_avg_5m"] = "0.1_0," + pyref.format_local(NOW0)
    ks.append(kat("E-underscore", a, -1, 90))
    a = anno_of([0.1] * 6)
    a["cpu_usage_avg_5m"] = "0.2," + pyref.format_local(NOW0).replace("Z", ".999999999Z")
    ks.append(kat("E-fraction", a, -1, 89, note="fractional seconds accepted after the seconds field"))
    a = anno_of([0.1] * 6)
    a["cpu_usage_avg_5m"] = "0.2,2026-02-30T20:00:00Z"
    ks.append(kat("E-baddate", a, -1, 81, note="day out of range"))
    ks.append(kat("E-daemonset", anno_of([1.5] * 6), -1, 0, ds=True, note="DaemonSet pods bypass Filter"))
    PE = dict(D)
    PE["priority"] = []
    ks.append(kat("E-noprio", anno_of([0.1] * 6, hv=2), -1, 0, policy=PE, note="no priorities: 0 - 20 -> clamp 0"))
    PS = dict(D)
    PS["syncPolicy"] = [("cpu_usage_avg_5m", 0)] + D["syncPolicy"][1:]
    ks.append(kat("E-nosync", anno_of([0.99, 0.1, 0.1, 0.1, 0.1, 0.1]), -1, 81, policy=PS,
                  note="period 0: predicate skipped, priority term 0 but weight counted"))
    # KAT-9: timestamp conversion
    t9 = pyref.go_parse_time("2026-10-15T20:00:00Z", "Asia/Shanghai")
    assert t9 == 1792065600 * 10**9
    times = {"KAT-9": {"s": "2026-10-15T20:00:00Z", "tz": "Asia/Shanghai", "unix_ns": t9}}
    # KAT-11: hot value
    pol = pyref.default_policy()
    bindings = [(0, NOW0 - s) for s in (0, 5, 10, 20, 30, 45, 59)] + [(0, NOW0 - s) for s in (61, 120, 200, 299)]
    bindings += [(0, NOW0 - 300), (1, NOW0 - 10), (7, NOW0 - 1)]  # 300s ago is outside 5m; node 7 absent
    cnts, hv = pyref.hot_values(pol, bindings, 4, NOW0)
    assert cnts[0][0] == 11 and cnts[1][0] == 7 and hv[0] == 5, (cnts, hv)
    hot = {"KAT-11": {"bindings": bindings, "n_nodes": 4, "now_unix": NOW0, "policy": policy_json(pol),
                      "expect_cnt": cnts, "expect_hv": hv}}
    floats = {}
    for s in ["0.5", "1_000.5", "_1", "1__0", "0x1p-2", "0x1", "+Inf", "-inf", "infinity", "infin", "NaN", "+NaN",
              "1e400", "1e-400", ".5", "5.", ".", "1e", "0x_1p0", " 1", "1 ", "", "1e1_0", "0.12345"]:
        v, err = pyref.go_parse_float(s)
        floats[s] = {"err": err, "value": None if err or v != v else (repr(v) if not (v in (float("inf"), float("-inf"))) else str(v)),
                     "nan": v != v}
    return {"kats": ks, "times": times, "hot": hot, "floats": floats}


def make_cluster(seed=20250216, n_nodes=64, n_pods=12):
    rng = random.Random(seed)
    pol = pyref.default_policy()
    nodes = []
    for n in range(n_nodes):
        a = {}
        for name, period in pol["syncPolicy"]:
            r = rng.random()
            if r < 0.06:
                continue  # missing
            dur_s = (period + pyref.EXTRA_ACTIVE_NS) // 10**9
            age = rng.randrange(0, int(1.5 * dur_s))
            u = round(rng.betavariate(2, 3) * 1.2, 5)
            v = f"{u:.5f}"
            if r < 0.08:
                v = "garbage"
            elif r < 0.09:
                v = f"-{u:.5f}"
            a[name] = f"{v},{pyref.format_local(NOW0 - age)}"
        if rng.random() < 0.9:
            a[pyref.NODE_HOT_VALUE] = f"{rng.randrange(0, 13)},{pyref.format_local(NOW0 - rng.randrange(0, 450))}"
        nodes.append(a)
    pods = []
    for p in range(n_pods):
        pods.append({"now_ns": NOW0_NS + p * 37_000_000_000, "daemonset": p == 5})
    ff, sc, ch = [], [], []
    for p in pods:
        fr, sr = [], []
        for a in nodes:
            fr.append(pyref.filter_node(pol, a, p["now_ns"], p["daemonset"]))
            sr.append(pyref.score_node(pol, a, p["now_ns"]))
        best, bs = -1, -1
        for i, (f, s) in enumerate(zip(fr, sr)):
            if f < 0 and s > bs:
                best, bs = i, s
        ff.append(fr)
        sc.append(sr)
        ch.append(best)
    return {"seed": seed, "tz": "Asia/Shanghai", "policy": policy_json(pol), "nodes": nodes, "pods": pods,
            "expect_filter": ff, "expect_score": sc, "expect_chosen": ch}


if __name__ == "__main__":
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(make_kats(), f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "cluster_small.json"), "w") as f:
        json.dump(make_cluster(), f, indent=1, sort_keys=True)
    print("wrote kats.json, cluster_small.json")
