"""Framework-level selection (crane_dyn_select, select.hip) against
the restatement in oracle/select.py of kube-scheduler v1.23.3's
numFeasibleNodesToFind / findNodesThatPassFilters / prioritizeNodes / selectHost
(generic_scheduler.go, not in the container: parity unpinned by reference tests)
with the shipped profile's Dynamic weight 3 (deploy/manifests/dynamic/
scheduler-config.yaml:13-15) and synthetic other-plugin filters and scores."""
import numpy as np
import pytest

from helpers import engine_for, oracle_soa

cd = pytest.importorskip("crane_dyn")
from crane_dyn import synth  # noqa: E402
from oracle import select as S  # noqa: E402


@pytest.mark.parametrize("n,pct,want", [
    (0, 0, 0), (50, 0, 50), (99, 10, 99), (100, 0, 100), (150, 10, 100), (1000, 0, 420), (1000, 30, 300),
    (5000, 0, 500), (100000, 0, 5000), (100000, 100, 100000), (100000, 120, 100000), (6250, 0, 312),
    (6249, 0, 312), (2000, -5, 680),
])
def test_num_feasible_nodes_to_find(n, pct, want):
    assert S.num_feasible_nodes_to_find(n, pct) == want
    assert cd.num_feasible_nodes_to_find(n, pct) == want


def test_oracle_select_rotation_and_ties():
    """The window walks the rotation: starts chain by the nodes checked; full windows
    when every node is scored; the seeded tie keys are a bijection of the node index."""
    rng = np.random.default_rng(1)
    P, N = 40, 400
    ff = np.where(rng.random((P, N)) < 0.2, 0, -1).astype(np.int8)
    sc = rng.integers(0, 3, (P, N))
    ds = np.zeros(P, np.uint8)
    ch, tot, ws, wl, nxt = S.framework_select(ff, sc, ds, percentage=0, start=17)
    K = S.num_feasible_nodes_to_find(N, 0)
    assert ws[0] == 17 and all(ws[p + 1] == (ws[p] + wl[p]) % N for p in range(P - 1))
    assert nxt == (ws[-1] + wl[-1]) % N
    for p in range(P):
        win = (ws[p] + np.arange(wl[p])) % N
        assert (ff[p, win] < 0).sum() == K and ff[p, win[-1]] < 0  # the window ends on the K-th feasible
    ch, tot, ws, wl, nxt = S.framework_select(ff, sc, ds, percentage=100, start=5)
    assert (ws == 5).all() and (wl == N).all() and nxt == 5
    for seed in (0, 7, 2**63 + 11):
        tk = S.tie_keys(seed, 5000, 3)
        assert len(np.unique(tk)) == 5000


def _cluster(N, P, seed, step_ns=1_000_000_000):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, N, P, seed=seed, pod_step_ns=step_ns, ds_frac=0.05)
    return spec, c


def _run(eng, c, ext_ok, ext_score, w, pct, start, seed):
    import torch
    dev = torch.device("cuda", 0)
    P = len(c.now)
    d_now = torch.from_numpy(c.now).to(dev)
    d_fl = torch.from_numpy(c.ds).to(dev)
    d_ok = None if ext_ok is None else torch.from_numpy(ext_ok.astype(np.uint8)).to(dev)
    d_ext = None if ext_score is None else torch.from_numpy(ext_score.astype(np.int64)).to(dev)
    ch = torch.empty(P, dtype=torch.int64, device=dev)
    tot = torch.empty(P, dtype=torch.int64, device=dev)
    ws = torch.empty(P, dtype=torch.int64, device=dev)
    wl = torch.empty(P, dtype=torch.int64, device=dev)
    nxt = eng.select(d_now, d_fl, ch, tot, d_ok, d_ext, dyn_weight=w, percentage=pct, start=start, tie_seed=seed,
                     d_wstart=ws, d_wlen=wl)
    torch.cuda.synchronize()
    return ch.cpu().numpy(), tot.cpu().numpy(), ws.cpu().numpy(), wl.cpu().numpy(), nxt


@pytest.mark.gpu
@pytest.mark.parametrize("N,P,pct,seed,start", [
    (3000, 300, 0, 0, 0),            # adaptive: 26 % -> 780 nodes per pod, rotating windows
    (3000, 300, 0, 987654321, 1234),  # seeded tie-break
    (2500, 200, 100, 0, 7),          # every node scored: no windows, start kept
    (64, 50, 0, 5, 3),               # N < 100: every node
    (1000, 257, 13, 0, 999),         # explicit percentage
])
def test_select_vs_oracle(N, P, pct, seed, start):
    spec, c = _cluster(N, P, seed=100 + N + P)
    rng = np.random.default_rng(N + P)
    ext_ok = rng.random(N) < 0.9
    # other plugins' weighted sum (7 default score plugins x 100), coarse so totals tie
    ext_score = rng.integers(0, 8, N) * 100
    off, osc, _ = oracle_soa(spec, c)
    want = S.framework_select(off, osc, c.ds, ext_ok, ext_score, 3, pct, start, seed)
    eng = engine_for(spec, c)
    got = _run(eng, c, ext_ok, ext_score, 3, pct, start, seed)
    eng.close()
    for name, g, w in zip(("chosen", "total", "wstart", "wlen"), got[:4], want[:4]):
        assert np.array_equal(g, w), (name, np.nonzero(g != w)[0][:5])
    assert got[4] == want[4]


@pytest.mark.gpu
def test_select_dynamic_only_matches_step_path():
    """Dynamic alone at weight 1, every node scored, lowest-index ties: the engine's own
    chosen node (the step / per-pair paths)."""
    spec, c = _cluster(4099, 513, seed=31)
    eng = engine_for(spec, c)
    _, _, ch, _ = eng.eval(c.now, c.ds)
    got = _run(eng, c, None, None, 1, 100, 0, 0)
    eng.close()
    assert np.array_equal(got[0], ch)


@pytest.mark.gpu
def test_select_nothing_feasible_and_daemonsets():
    """Other filters reject every node: Unschedulable (-1), every node checked, the
    start advances by N (unchanged); DaemonSet pods still obey the other filters."""
    spec, c = _cluster(800, 100, seed=41)
    eng = engine_for(spec, c)
    none_ok = np.zeros(800, bool)
    got = _run(eng, c, none_ok, None, 3, 0, 11, 0)
    assert (got[0] == -1).all() and (got[1] == -1).all() and (got[3] == 800).all() and got[4] == 11
    c.ds[:] = 1
    ok = np.zeros(800, bool)
    ok[::7] = True
    off, osc, _ = oracle_soa(spec, c)
    want = S.framework_select(off, osc, c.ds, ok, None, 3, 0, 11, 0)
    got = _run(eng, c, ok, None, 3, 0, 11, 0)
    eng.close()
    for g, w in zip(got[:4], want[:4]):
        assert np.array_equal(g, w)
    assert got[4] == want[4]


def _bench_queue_ext(N):
    """The bench's config-3 selection leg's other-plugin verdicts (bench.py select_leg)."""
    rng = np.random.default_rng(77)
    return rng.random(N) < 0.95, rng.integers(0, 8, N).astype(np.int64) * 100


@pytest.mark.gpu
@pytest.mark.slow
def test_select_config3_queue_prefix():
    """The bench's config-3 queue (100k nodes x 10k pods, shipped profile, adaptive 5 %
    windows): the first 64 pods' windows, chosen nodes and totals equal the oracle's (a
    window chain's prefix depends on the queue's prefix only), and every pod's window
    equals the streaming chain kernel's (sel_chain 1)."""
    spec = cd.default_policy_spec()
    cfg = synth.CONFIGS[3]
    c = synth.make_cluster(spec, cfg["nodes"], cfg["pods"], n_bindings=0, seed=20250215 + 3000)
    c.now, c.ds = synth.make_pods(cfg["pods"], seed=20250215 + 3)
    ok, ext = _bench_queue_ext(c.n_nodes)
    eng = engine_for(spec, c)
    got = _run(eng, c, ok, ext, 3, 0, 0, 0)
    eng.set_option("sel_chain", 1)
    ref = _run(eng, c, ok, ext, 3, 0, 0, 0)
    eng.close()
    for name, g, r in zip(("chosen", "total", "wstart", "wlen"), got[:4], ref[:4]):
        assert np.array_equal(g, r), (name, np.nonzero(g != r)[0][:5])
    assert got[4] == ref[4]
    n = 64
    off, osc, _ = oracle_soa(spec, c, now=c.now[:n], ds=c.ds[:n])
    want = S.framework_select(off, osc, c.ds[:n], ok, ext, 3, 0, 0, 0)
    for name, g, w in zip(("chosen", "total", "wstart", "wlen"), got[:4], want[:4]):
        assert np.array_equal(g[:n], w), (name, np.nonzero(g[:n] != w)[0][:5])
    assert want[4] == (got[2][n] if len(got[2]) > n else got[4])


@pytest.mark.gpu
@pytest.mark.parametrize("N,P,step_ns,pct", [(3000, 400, 1_000_000_000, 0), (20_000, 600, 60_000_000_000, 0),
                                             (131_072, 300, 1_000_000_000, 0), (131_073, 100, 1_000_000_000, 0),
                                             (5000, 700, 10_000_000, 2)])
def test_select_chain_forms_agree(N, P, step_ns, pct):
    """The LDS rank/select walk equals the streaming chain kernel pod for pod: few and many
    in-range nodes (pods minutes apart put more than its list holds in range: the streaming
    kernel then runs behind it), the size limit (131,072 nodes) and one past it, tiny
    windows."""
    spec, c = _cluster(N, P, seed=N + P, step_ns=step_ns)
    rng = np.random.default_rng(N)
    ok = rng.random(N) < 0.9
    eng = engine_for(spec, c)
    got = _run(eng, c, ok, None, 3, pct, 7, 0)
    eng.set_option("sel_chain", 1)
    ref = _run(eng, c, ok, None, 3, pct, 7, 0)
    eng.close()
    for name, g, r in zip(("chosen", "total", "wstart", "wlen"), got[:4], ref[:4]):
        assert np.array_equal(g, r), (name, np.nonzero(g != r)[0][:5])
    assert got[4] == ref[4]


@pytest.mark.gpu
@pytest.mark.parametrize("N,P,step_ns,pct,ds_frac,ok_frac,start", [
    (2000, 1500, 1_000_000_000, 0, 0.0, 0.9, 0),          # many rotations, no DaemonSet pods
    (2000, 1500, 1_000_000_000, 0, 0.3, 0.9, 1999),       # DaemonSet pods between rank-space runs
    (5000, 800, 20_000_000_000, 1, 0.1, 0.95, 4321),      # tiny windows, many in-range nodes
    (777, 900, 5_000_000_000, 40, 0.05, 0.6, 13),         # windows near the A count
    (3000, 400, 1_000_000_000, 60, 0.2, 0.3, 5),          # fewer A nodes than a window: position walk
    (64 * 300 + 17, 700, 2_000_000_000, 0, 1.0, 0.8, 9),  # every pod a DaemonSet pod
])
def test_select_rank_walk_agrees(N, P, step_ns, pct, ds_frac, ok_frac, start):
    """The rank-space walk (window ends as A ranks / I indices, positions resolved after the
    chain) equals the streaming chain kernel pod for pod, across DaemonSet mixes, window
    sizes, wrap-arounds over many rotations and the position-walk fallback."""
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, N, P, seed=N * 7 + P, pod_step_ns=step_ns, ds_frac=ds_frac)
    rng = np.random.default_rng(N + 1)
    ok = rng.random(N) < ok_frac
    eng = engine_for(spec, c)
    got = _run(eng, c, ok, None, 3, pct, start, 0)
    eng.set_option("sel_chain", 1)
    ref = _run(eng, c, ok, None, 3, pct, start, 0)
    eng.close()
    for name, g, r in zip(("chosen", "total", "wstart", "wlen"), got[:4], ref[:4]):
        assert np.array_equal(g, r), (name, np.nonzero(g != r)[0][:5])
    assert got[4] == ref[4]
    if N <= 3000 and P <= 900:
        off, osc, _ = oracle_soa(spec, c)
        want = S.framework_select(off, osc, c.ds, ok, None, 3, pct, start, 0)
        for name, g, w in zip(("chosen", "total", "wstart", "wlen"), got[:4], want[:4]):
            assert np.array_equal(g, w), (name, np.nonzero(g != w)[0][:5])
