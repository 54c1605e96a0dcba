"""Sequential-greedy placement (crane_dyn_greedy) vs the oracle's or_greedy.

Each placement is a Binding{Timestamp: now} on the chosen node, which raises
its window counts / hot value (binding.go:81-97, node.go:113-121) before the
next pod is scored (plugins.go:73-98).  Bit-exact chosen nodes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

cd = pytest.importorskip("crane_dyn")
from crane_dyn import synth  # noqa: E402
from helpers import engine_for  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _oracle(spec, c, P, now):
    return O.greedy(spec, c.metric_names, c.ok, c.val, np.where(c.ok == 1, c.ts, 0), c.b_node, c.b_ts, now, P,
                    c.ds[:P])


@pytest.mark.parametrize("N,P,B,seed", [(1, 5, 0, 1), (64, 200, 1000, 2), (1000, 3000, 20000, 3),
                                        (4097, 2000, 50000, 4), (20000, 5000, 200000, 5)])
def test_greedy_vs_oracle(N, P, B, seed):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, N, P, n_bindings=B, seed=seed, ds_frac=0.05)
    now = int(synth.NOW0_NS) + 1234567
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    ch = eng.greedy(P, now, c.ds)
    och = _oracle(spec, c, P, now)
    assert np.array_equal(ch, och)


def test_greedy_global_leaves():
    """N above the LDS leaf capacity: leaves stay in global memory."""
    spec = cd.default_policy_spec()
    N, P = 200_000, 3000
    c = synth.make_cluster(spec, N, P, n_bindings=100_000, seed=9)
    now = int(synth.NOW0_NS)
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    ch = eng.greedy(P, now, c.ds)
    assert np.array_equal(ch, _oracle(spec, c, P, now))


def test_greedy_edge_policies():
    m = 60 * 10**9
    base = cd.default_policy_spec()
    specs = [dict(base, priority=[]), dict(base, hotValue=[]), dict(base, hotValue=[(0, 1), (-60 * m, 2), (30 * m, -3)])]
    for i, spec in enumerate(specs):
        c = synth.make_cluster(spec, 300, 400, n_bindings=5000, seed=40 + i)
        now = int(synth.NOW0_NS)
        eng = engine_for(spec, c)
        eng.upload_bindings(c.b_node, c.b_ts)
        ch = eng.greedy(400, now, c.ds)
        assert np.array_equal(ch, _oracle(spec, c, 400, now)), i


def test_greedy_then_eval_consistent():
    """greedy leaves the engine usable: a later eval recomputes node records."""
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 500, 50, n_bindings=3000, seed=8)
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    eng.greedy(50, int(c.now[0]), c.ds)
    eng.upload_nodes(*c.rows(eng.metric_names)[:2], c.hv, c.hv_ts)
    _, _, ch, _ = eng.eval(c.now, c.ds)
    from helpers import oracle_soa
    assert np.array_equal(ch, oracle_soa(spec, c, want_matrix=False)[2])
