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
