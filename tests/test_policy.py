"""Strict DynamicSchedulerPolicy decoding (crane_policy_load_*), the C++ restatement of
LoadPolicyFromFile/loadPolicy (pkg/plugins/dynamic/policyfile.go:11-33) with the strict
codec of pkg/plugins/apis/policy/scheme/scheme.go:17 and the v1alpha1 JSON names of
pkg/plugins/apis/policy/v1alpha1/types.go:14-39."""
import json
import os

import pytest

from conftest import GOLDEN

cd = pytest.importorskip("crane_dyn")
from oracle import oracle as O  # noqa: E402

DEFAULT = os.path.join(GOLDEN, "policy_default.yaml")
HDR = "apiVersion: scheduler.policy.crane.io/v1alpha1\nkind: DynamicSchedulerPolicy\n"


def test_default_policy_file():
    p = cd.Policy.load_file(DEFAULT)
    assert p.spec == {k: [tuple(x) for x in v] for k, v in cd.default_policy_spec().items()}


REF_POLICY = "/root/reference/deploy/manifests/dynamic/policy.yaml"


@pytest.mark.skipif(not os.path.exists(REF_POLICY), reason="reference checkout absent (build container only)")
def test_reference_policy_file():
    """The reference's own shipped policy (deploy/manifests/dynamic/policy.yaml:1-52), read in
    place with its '##' comment lines and blank lines, decodes to the default policy — the one
    datum on this path the reference itself holds.  The fixture copy must decode the same."""
    p = cd.Policy.load_file(REF_POLICY)
    assert p.spec == {k: [tuple(x) for x in v] for k, v in cd.default_policy_spec().items()}
    assert p.spec == cd.Policy.load_file(DEFAULT).spec
    with open(REF_POLICY, "rb") as f:
        assert cd.Policy.load_bytes(f.read()).spec == p.spec


def test_json_equivalent():
    spec = cd.default_policy_spec()
    m = 60 * 10**9
    dur = {3 * m: "3m", 15 * m: "15m", 180 * m: "3h", 5 * m: "5m", 1 * m: "1m"}
    doc = {"apiVersion": "scheduler.policy.crane.io/v1alpha1", "kind": "DynamicSchedulerPolicy", "spec": {
        "syncPolicy": [{"name": n, "period": dur[p]} for n, p in spec["syncPolicy"]],
        "predicate": [{"name": n, "maxLimitPecent": v} for n, v in spec["predicate"]],
        "priority": [{"name": n, "weight": v} for n, v in spec["priority"]],
        "hotValue": [{"timeRange": dur[t], "count": c} for t, c in spec["hotValue"]]}}
    assert cd.Policy.load_bytes(json.dumps(doc)).spec == cd.Policy.load_file(DEFAULT).spec


@pytest.mark.parametrize("body,match", [
    ("spec:\n  syncPolicy:\n  - name: a\n    period: 3m\n    extra: 1\n", "unknown field"),
    ("spec:\n  predicate:\n  - name: a\n    name: b\n", "duplicate field"),
    ("spec:\n  syncPolicy:\n  - name: a\n    period: 3q\n", "invalid duration"),
    ("spec:\n  syncPolicy:\n  - name: a\n    period: 180\n", "Duration"),
    ("spec:\n  hotValue:\n  - timeRange: 5m\n    count: 5.0\n", "into int"),
    ("spec:\n  priority:\n  - name: a\n    weight: heavy\n", "float64"),
    ("spec:\n  predicate:\n  - name: 12\n", "into string"),
    ("metadata:\n  name: x\n", "unknown field"),
    ("spec:\n  priorities: []\n", "unknown field"),
])
def test_strict_errors(body, match):
    with pytest.raises(cd.CraneError, match=match):
        cd.Policy.load_bytes(HDR + body)


def test_kind_and_version():
    with pytest.raises(cd.CraneError, match="Kind"):
        cd.Policy.load_bytes("apiVersion: scheduler.policy.crane.io/v1alpha1\nspec: {}\n")
    with pytest.raises(cd.CraneError, match="registered"):
        cd.Policy.load_bytes("apiVersion: v1\nkind: DynamicSchedulerPolicy\n")
    with pytest.raises(cd.CraneError) as e:
        cd.Policy.load_file("/nonexistent/policy.yaml")
    assert e.value.code == -5


def test_yaml_forms():
    p = cd.Policy.load_bytes(HDR + """spec:
  syncPolicy:
  - name: "quoted"   # comment
    period: '1h30m'
  predicate: []
  priority:
  -
    name: x
    weight: 1e-1
  hotValue: ~
""")
    assert p.spec["syncPolicy"] == [("quoted", 5400 * 10**9)]
    assert p.spec["predicate"] == [] and p.spec["hotValue"] == []
    assert p.spec["priority"] == [("x", 0.1)]


@pytest.mark.parametrize("d", ["3m", "15m", "3h", "1h30m", "1.5h", "300ms", "-5m", "0", "2µs", "1.001s", "0.5h", "12ns"])
def test_durations_match_oracle(d):
    p = cd.Policy.load_bytes(HDR + f"spec:\n  syncPolicy:\n  - name: a\n    period: \"{d}\"\n")
    assert p.spec["syncPolicy"][0][1] == O.go_parse_duration(d)
