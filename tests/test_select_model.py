"""The rank-space selection walk's bookkeeping (k_sel_chain_rs, select.hip) on the CPU: a
lane-level model of the kernel's chain (tools/select_rank_walk_model.py) against a
brute-force position walk, random queues with DaemonSet pods, in-range nodes, windows
from 1 node to every always-feasible node, and list lengths below a wave (the cached
entries then span several rotations)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import select_rank_walk_model as M  # noqa: E402


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_rank_walk_model_matches_position_walk(seed):
    assert M.main(seed, trials=60) == 0
