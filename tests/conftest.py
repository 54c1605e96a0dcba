"""Shared pytest setup: markers, import paths, fixture loaders."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "crane-scheduler_amd"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: full-size parity runs (GPU)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def policy_from_json(p):
    return {"syncPolicy": [(n, int(v)) for n, v in p["syncPolicy"]],
            "predicate": [(n, float(v)) for n, v in p["predicate"]],
            "priority": [(n, float(v)) for n, v in p["priority"]],
            "hotValue": [(int(t), int(c)) for t, c in p["hotValue"]]}


@pytest.fixture(scope="session")
def kats():
    return load_golden("kats.json")


@pytest.fixture(scope="session")
def cluster_small():
    return load_golden("cluster_small.json")
