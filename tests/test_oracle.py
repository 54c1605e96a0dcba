"""The CPU oracle (oracle/crane_oracle.c) against the committed golden vectors.

Both restatements — the C oracle and tests/golden/pyref.py — follow
/root/reference/pkg/plugins/dynamic/stats.go + plugins.go; the KATs pin the
hand-derived values of SURVEY.md §8c.
"""
import math

import numpy as np
import pytest

from conftest import policy_from_json
from oracle import oracle as O

SH = 8 * 3600  # Asia/Shanghai, UTC+8


def test_kat_filter_score_strings(kats):
    for k in kats["kats"]:
        pol = policy_from_json(k["policy"])
        ff, sc, ch = O.eval_strings(pol, [k["annotations"]], [k["now_ns"]], [k["daemonset"]])
        assert ff[0, 0] == k["expect_filter"], k["name"]
        assert sc[0, 0] == k["expect_score"], k["name"]
        assert ch[0] == (0 if k["expect_filter"] < 0 else -1), k["name"]


def test_kat_time(kats):
    t = kats["times"]["KAT-9"]
    assert O.go_parse_time(t["s"], SH) == t["unix_ns"] == 1792065600 * 10**9


def test_kat_floats(kats):
    for s, e in kats["floats"].items():
        v, err = O.go_parse_float(s)
        assert err == e["err"], s
        if err is None:
            if e["nan"]:
                assert math.isnan(v), s
            else:
                assert v == float(e["value"]), s


def test_kat_hot_value(kats):
    h = kats["hot"]["KAT-11"]
    pol = policy_from_json(h["policy"])
    b = np.array(h["bindings"], np.int64)
    cnt, hv = O.hot_values(pol, b[:, 0], b[:, 1], h["n_nodes"], h["now_unix"])
    assert cnt.tolist() == h["expect_cnt"]
    assert hv.tolist() == h["expect_hv"]
    assert hv[0] == 5  # SURVEY KAT-11: 11/5 + 7/2 = 2 + 3


def test_golden_cluster_strings(cluster_small):
    c = cluster_small
    pol = policy_from_json(c["policy"])
    now = [p["now_ns"] for p in c["pods"]]
    ds = [p["daemonset"] for p in c["pods"]]
    for threads in (1, 4):
        ff, sc, ch = O.eval_strings(pol, c["nodes"], now, ds, threads=threads)
        assert ff.tolist() == c["expect_filter"]
        assert sc.tolist() == c["expect_score"]
        assert ch.tolist() == c["expect_chosen"]


def test_golden_cluster_soa_matches_strings(cluster_small):
    """SoA mode (pre-parsed once) == string mode (re-parsed per call)."""
    c = cluster_small
    pol = policy_from_json(c["policy"])
    keys = [n for n, _ in pol["syncPolicy"]]
    N = len(c["nodes"])
    ok = np.zeros((len(keys), N), np.uint8)
    val = np.zeros((len(keys), N))
    ts = np.zeros((len(keys), N), np.int64)
    hv_ok = np.zeros(N, np.uint8)
    hv = np.zeros(N)
    hv_ts = np.zeros(N, np.int64)
    for n, a in enumerate(c["nodes"]):
        for k, name in enumerate(keys):
            if name in a:
                ok[k, n], val[k, n], ts[k, n] = O.parse_annotation(a[name], SH)
        if "node_hot_value" in a:
            hv_ok[n], hv[n], hv_ts[n] = O.parse_annotation(a["node_hot_value"], SH)
    now = [p["now_ns"] for p in c["pods"]]
    ds = [p["daemonset"] for p in c["pods"]]
    ff, sc, ch = O.eval_soa(pol, keys, ok, val, ts, hv_ok, hv, hv_ts, now, ds)
    assert ff.tolist() == c["expect_filter"]
    assert sc.tolist() == c["expect_score"]
    assert ch.tolist() == c["expect_chosen"]


@pytest.mark.parametrize("s,ns", [("3m", 180 * 10**9), ("15m", 900 * 10**9), ("3h", 10800 * 10**9),
                                  ("1h30m", 5400 * 10**9), ("1.5h", 5400 * 10**9), ("300ms", 3 * 10**8),
                                  ("-5m", -300 * 10**9), ("0", 0), ("2µs", 2000), ("1.001s", 1001 * 10**6)])
def test_parse_duration(s, ns):
    assert O.go_parse_duration(s) == ns


@pytest.mark.parametrize("s", ["", "3", "m", "3x", "1.s.", ".s", "+", "1h 2m"])
def test_parse_duration_bad(s):
    assert O.go_parse_duration(s) is None


def test_go_f64_to_int():
    assert O.go_f64_to_int(float("nan")) == -(2**63)
    assert O.go_f64_to_int(float("inf")) == -(2**63)
    assert O.go_f64_to_int(-float("inf")) == -(2**63)
    assert O.go_f64_to_int(9.3e18) == -(2**63)
    assert O.go_f64_to_int(-9.2e18) == -9200000000000000000
    assert O.go_f64_to_int(48.99999999999999) == 48
    assert O.go_f64_to_int(-0.9) == 0


def test_time_edge_cases():
    assert O.go_parse_time("2026-10-15T20:00:00Z", 0) == 1792094400 * 10**9
    assert O.go_parse_time("2026-10-15T7:00:00Z", 0) is not None  # stdHour accepts one digit
    assert O.go_parse_time("2026-1-15T07:00:00Z", 0) is None  # stdZeroMonth needs two
    assert O.go_parse_time("2024-02-29T00:00:00Z", 0) is not None
    assert O.go_parse_time("2023-02-29T00:00:00Z", 0) is None
    assert O.go_parse_time("2026-10-15T24:00:00Z", 0) is None
    assert O.go_parse_time("2026-10-15T20:00:00", 0) is None
    assert O.go_parse_time("2026-10-15T20:00:00.5Z", 0) == 1792094400 * 10**9 + 500_000_000
    assert O.go_parse_time("2026-10-15T20:00:00.1234567891Z", 0) == 1792094400 * 10**9 + 123456789
