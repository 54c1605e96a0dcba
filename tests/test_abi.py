"""CPU-side checks of the C ABI library: it loads, exports every declared symbol,
and its host-only pieces (annotation parser, policy decoder) match the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import oracle as O

cd = pytest.importorskip("crane_dyn")


def test_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "crane_dyn.h")).read()
    declared = set(re.findall(r"\b(crane_\w+)\s*\(", hdr))
    lib = ctypes.CDLL(cd.LIB_PATH)
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == set(cd.ABI_SYMBOLS)


def test_parse_annotation_matches_oracle(kats, cluster_small):
    strs = set()
    for k in kats["kats"]:
        strs.update(k["annotations"].values())
    for a in cluster_small["nodes"]:
        strs.update(a.values())
    strs.update(["", ",", "1,2", "0.5,2026-10-15T20:00:00Z", "0.5,2026-10-15T20:00:00.123Z", "0x1p-1,2026-10-15T20:00:00Z",
                 "1_0,2026-10-15T20:00:00Z", "inf,2026-10-15T20:00:00Z", "nan,2026-10-15T20:00:00Z",
                 "+nan,2026-10-15T20:00:00Z", "1e999,2026-10-15T20:00:00Z", "0.5,2026-13-15T20:00:00Z"])
    for s in sorted(strs):
        v, ts = cd.parse_annotation(s, 8 * 3600)
        ok, ov, ots = O.parse_annotation(s, 8 * 3600)
        assert (ts != cd.CRANE_TS_INVALID) == ok, s
        if ok:
            assert ts == ots, s
            assert (v == ov) or (v != v and ov != ov), s


def test_tz_offsets(monkeypatch):
    assert cd.tz_offset("Asia/Shanghai") == 8 * 3600
    assert cd.tz_offset("UTC") == 0
    assert cd.tz_offset("Etc/GMT-8") == 8 * 3600
    monkeypatch.delenv("TZ", raising=False)
    assert cd.tz_offset(None) == 8 * 3600  # utils.DefaultTimeZone
    with pytest.raises(cd.CraneError):
        cd.tz_offset("Mars/Olympus")


def test_key_decode():
    assert cd.key_node(-1) == (-1, -1)
    key = (87 << 32) | (0xFFFFFFFF - 12345)
    assert cd.key_node(key) == (12345, 87)


def test_engine_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(cd.CraneError):
        cd.Engine(cd.Policy(cd.default_policy_spec()))


def test_engine_rejects_bad_policy():
    spec = cd.default_policy_spec()
    spec["hotValue"] = [(60 * 10**9, 0)]
    with pytest.raises(cd.CraneError, match="count"):
        cd.Engine(cd.Policy(spec))


def test_bulk_parse_matches_single(cluster_small):
    nodes = cluster_small["nodes"] * 50
    names = ["cpu_usage_avg_5m", "cpu_usage_max_avg_1h", "cpu_usage_max_avg_1d", "mem_usage_avg_5m",
             "mem_usage_max_avg_1h", "mem_usage_max_avg_1d"]
    val, ts, hv, hv_ts = cd.parse_nodes(names, nodes, 8 * 3600)
    for n in range(0, len(nodes), 37):
        for m, k in enumerate(names):
            if k in nodes[n]:
                v1, t1 = cd.parse_annotation(nodes[n][k], 8 * 3600)
                assert t1 == ts[m, n] and (v1 == val[m, n] or (v1 != v1 and val[m, n] != val[m, n]))
            else:
                assert ts[m, n] == cd.CRANE_TS_INVALID
        if "node_hot_value" in nodes[n]:
            assert (hv[n], hv_ts[n]) == cd.parse_annotation(nodes[n]["node_hot_value"], 8 * 3600)


def test_snapshot_parse_matches_generator_soa():
    """Bulk parse of a synthetic snapshot's annotation strings reproduces the generator's own
    SoA: well-formed values bit-exact, missing/malformed keys CRANE_TS_INVALID, negatives kept
    (the engine rejects them like stats.go:71-73); thread count does not change the result."""
    from crane_dyn import synth
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 12000, 1, seed=7)  # 84k strings: 2 threads of >= 32k
    snap = cd.SnapshotStrings(c.metric_names, c.annotations())
    snap.parse(synth.SHANGHAI, threads=1)
    val, ts, hv, hv_ts = snap.soa()
    snap.parse(synth.SHANGHAI, threads=4)
    v4, t4, _, _ = snap.soa()
    assert np.array_equal(ts, t4) and np.array_equal(val.view(np.int64), v4.view(np.int64))
    ok = c.ok.astype(bool)
    assert np.array_equal(ts[ok], c.ts[ok]) and np.array_equal(val[ok], c.val[ok])
    assert (ts[~ok] == cd.CRANE_TS_INVALID).all()
    assert (val[ok] < 0).any()
    assert np.array_equal(hv, c.hv) and np.array_equal(hv_ts, c.hv_ts)


def test_parse_float_fast_path_matches_correct_rounding():
    """The decimal fast path (mantissa <= 2^53, <= 22 fraction digits) must return the
    correctly rounded double, i.e. what strconv.ParseFloat (and Python's float) return."""
    rng = np.random.default_rng(11)
    cases = ["0", "-0", "+7", "1.", "0.00000", "-0.00000", "9007199254740992", "9007199254740993",
             "0.1", "0.30000", "1.23456789012345678", "123456789012345678901", "1e5", ".5", "-.5",
             "4503599627370497.5", "0.0000000000000000000001", "0.00000000000000000000001"]
    cases += [f"{x:.5f}" for x in rng.random(2000) * 1.2]
    cases += [f"{x:.{k}f}" for x, k in zip(rng.random(2000) * 10.0 ** rng.integers(0, 12, 2000),
                                           rng.integers(0, 23, 2000))]
    cases += [str(int(x)) for x in rng.integers(0, 2**62, 500)]
    for s in cases:
        v, t = cd.parse_annotation(s + ",2026-10-15T20:00:00Z", 8 * 3600)
        assert t == 1792065600 * 10**9, s
        want = float(s)
        assert v == want and np.signbit(v) == np.signbit(want), (s, v, want)


def test_parse_time_fixed_layout_matches_oracle():
    """The 20-byte stamp fast path (fixed positions, per-thread date memo) against the oracle's
    general ParseInLocation restatement: random fields in and out of range, far years
    (saturated ns), corrupted bytes, and repeated dates in one bulk parse (the memo)."""
    rng = np.random.default_rng(5)
    strs = []
    for _ in range(3000):
        y = int(rng.choice([rng.integers(0, 10000), rng.integers(1990, 2100)]))
        f = [y, rng.integers(0, 14), rng.integers(0, 33), rng.integers(0, 26), rng.integers(0, 62),
             rng.integers(0, 62)]
        s = "%04d-%02d-%02dT%02d:%02d:%02dZ" % tuple(int(x) for x in f)
        if rng.random() < 0.1:
            i = int(rng.integers(0, 20))
            s = s[:i] + chr(int(rng.integers(32, 127))) + s[i + 1:]
        strs.append("0.5," + s)
    strs += ["0.5,2024-02-29T00:00:00Z", "0.5,2023-02-29T00:00:00Z", "0.5,2023-02-28T23:59:59Z"] * 3
    # the memo key of an out-of-range day must not alias the next month's day 1 .. 3:
    # (2026, 1, 33) once keyed like (2026, 2, 1)
    strs += ["0.5,2026-02-01T00:00:00Z", "0.5,2026-01-33T00:00:00Z", "0.5,2026-01-32T00:00:00Z",
             "0.5,2026-03-02T00:00:00Z", "0.5,2026-02-34T00:00:00Z", "0.5,2026-01-00T00:00:00Z"]
    nodes = [{"m": s} for s in strs]
    val, ts, _, _ = cd.parse_nodes(["m"], nodes, 8 * 3600, threads=1)
    for n, s in enumerate(strs):
        ok, _, ots = O.parse_annotation(s, 8 * 3600)
        assert (ts[0, n] != cd.CRANE_TS_INVALID) == ok, s
        if ok:
            assert ts[0, n] == ots, s
