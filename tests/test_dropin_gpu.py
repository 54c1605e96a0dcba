"""Incremental drop-in updates (crane_dyn_update_nodes + crane_dyn_node_steps_subset, and the
fused crane_dyn_update_node_steps).

The reference plugin reads the node's CURRENT annotations on every Filter / Score call
(/root/reference/pkg/plugins/dynamic/stats.go:51-76) while the controller patches them
continuously: every (node, metric) sync writes the metric and node_hot_value
(pkg/controller/annotator/node.go:88-96,123-146) at each syncPolicy period
(node.go:148-177).  The engine takes those patches as scatter updates of the changed
nodes, and the plugin's answer table is patched row by row.  After many rounds of
updates the patched table must equal a full rebuild on the same engine, a fresh engine
holding the final snapshot, and the oracle's per-call answers."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

cd = pytest.importorskip("crane_dyn")
from crane_dyn import synth  # noqa: E402
from helpers import engine_for, oracle_soa  # noqa: E402

TS_INVALID = synth.TS_INVALID


def churn(c, spec, rng, idx, now_ns, hv_present=True):
    """New annotations on nodes idx of cluster c (in place), as the controller writes them
    at now_ns: fresh metric values (5-decimal domain, prometheus.go:124), stamps up to 1.5
    active periods old, some missing / malformed / negative, hot value 0..12."""
    periods = dict(spec["syncPolicy"])
    k = len(idx)
    for m, name in enumerate(c.metric_names):
        dur_s = (periods[name] + 300 * 10**9) // 10**9
        v = np.round(rng.beta(2.0, 3.0, k) * 1.2 * 1e5) / 1e5
        age = np.floor(rng.random(k) * 1.5 * dur_s).astype(np.int64)
        ts = (now_ns // 10**9 - age) * 10**9
        r = rng.random(k)
        bad = r < 0.05
        v = np.where((r >= 0.05) & (r < 0.07), -np.maximum(v, 1e-5), v)
        c.ok[m, idx] = np.where(bad, 0, 1)
        c.val[m, idx] = np.where(bad, 0.0, v)
        c.ts[m, idx] = np.where(bad, TS_INVALID, ts)
    if hv_present:
        c.hv[idx] = rng.integers(0, 13, k).astype(np.float64)
        c.hv_ts[idx] = (now_ns // 10**9 - rng.integers(0, 450, k)) * 10**9
        c.hv_ts[idx[rng.random(k) < 0.05]] = TS_INVALID
    else:
        c.hv[idx] = 0.0
        c.hv_ts[idx] = TS_INVALID


def push(eng, c, idx, hv_present=True):
    val, ts, _ = c.rows(eng.metric_names)
    if hv_present:
        eng.update_nodes(idx, val[:, idx], ts[:, idx], c.hv[idx], c.hv_ts[idx])
    else:
        eng.update_nodes(idx, val[:, idx], ts[:, idx])


def patch(tab, rows, idx):
    for full, part in zip(tab, rows):
        full[idx] = part


def same_tables(a, b):
    """Equal answer tables: breakpoint counts, the live breakpoints and their values."""
    ns_a, ns_b = a[0], b[0]
    if not np.array_equal(ns_a, ns_b):
        return False
    S = a[1].shape[1]
    live_bp = np.arange(S)[None, :] < ns_a[:, None]
    live_v = np.arange(S + 1)[None, :] <= ns_a[:, None]
    return (np.array_equal(np.where(live_bp, a[1], 0), np.where(live_bp, b[1], 0))
            and np.array_equal(np.where(live_v, a[2], 0), np.where(live_v, b[2], 0))
            and np.array_equal(np.where(live_v, a[3], 0), np.where(live_v, b[3], 0)))


@pytest.mark.parametrize("N,seed", [(20_000, 41), (777, 42)])
def test_incremental_tables_equal_rebuild_and_oracle(N, seed):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, N, 4, seed=seed)
    eng = engine_for(spec, c)
    t0 = int(synth.NOW0_NS) - 3 * 10**9
    t1 = t0 + 60 * 10**9
    tab = [x.copy() for x in eng.node_steps(t0, t1)]
    rng = np.random.default_rng(seed)
    now = int(synth.NOW0_NS)
    for r, k in enumerate([1, 3, 17, 300, 2, min(N, 1500), 5, 64, 1, 9, 33, 250]):
        idx = rng.choice(N, size=k, replace=False).astype(np.int64)
        hv_present = r != 6  # one round of patches without node_hot_value on those nodes
        now += int(rng.integers(1, 400)) * 10**6
        churn(c, spec, rng, idx, now, hv_present)
        if r % 2:  # the fused form: columns, records and rows in one call
            val, ts, _ = c.rows(eng.metric_names)
            hv, hv_ts = (c.hv[idx], c.hv_ts[idx]) if hv_present else (None, None)
            patch(tab, eng.update_node_steps(idx, val[:, idx], ts[:, idx], hv, hv_ts, t0, t1), idx)
        else:
            push(eng, c, idx, hv_present)
            patch(tab, eng.node_steps_subset(t0, t1, idx), idx)
        if r in (0, 5, 11):  # the same engine's full table over its updated records
            assert same_tables(tab, eng.node_steps(t0, t1)), r
    fresh = engine_for(spec, c)  # one full upload of the final snapshot (K1's records)
    assert same_tables(tab, fresh.node_steps(t0, t1))
    # the oracle's per-call answers at pod times across the horizon, breakpoints included
    ns, bp = tab[0], tab[1]
    bps = np.unique(np.concatenate([bp[i, :ns[i]] for i in range(N)] + [np.array([t0], np.int64)]))
    pick = rng.choice(bps, min(8, len(bps)), replace=False)
    times = np.unique(np.concatenate([pick, pick - 1, [t0, t1 - 1]]))
    times = times[(times >= t0) & (times < t1)]
    off, osc, _ = oracle_soa(spec, c, now=times.astype(np.int64), ds=np.zeros(len(times), np.uint8))
    for j, t in enumerate(times):
        ff, sc = cd.Engine.table_lookup(tab, int(t))
        assert np.array_equal(ff, off[j]) and np.array_equal(sc, osc[j]), int(t)
    # the batched paths read the scattered SoA: keys / matrices equal the fresh engine's
    pods = np.sort(rng.integers(t0, t1, 40)).astype(np.int64)
    ds = (rng.random(40) < 0.1).astype(np.uint8)
    a = eng.eval(pods, ds, matrix=True, compact=True)
    b = fresh.eval(pods, ds, matrix=True, compact=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    eng.close()
    fresh.close()


def test_update_after_binding_hot_values():
    """After a refresh from the binding log the hot values come from counts; an update
    returns the shard to annotation hot values, like a full upload does."""
    spec = cd.default_policy_spec()
    N = 5000
    c = synth.make_cluster(spec, N, 16, n_bindings=50_000, seed=43)
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    now = int(synth.NOW0_NS)
    eng.refresh_hot_values(now, now)
    _ = eng.eval(c.now[:2], c.ds[:2])  # records built from the counts
    rng = np.random.default_rng(43)
    idx = rng.choice(N, 40, replace=False).astype(np.int64)
    churn(c, spec, rng, idx, now + 5 * 10**9)
    push(eng, c, idx)
    fresh = engine_for(spec, c)
    for x, y in zip(eng.eval(c.now, c.ds, matrix=True), fresh.eval(c.now, c.ds, matrix=True)):
        assert np.array_equal(x, y)
    assert np.array_equal(eng.hot_values(), c.hv)
    eng.close()
    fresh.close()


def test_update_shard_without_hot_value_annotations():
    """A shard uploaded with no node_hot_value (hv NULL) that then receives some: the other
    nodes keep none (0, unusable), as a full upload of the same snapshot gives."""
    spec = cd.default_policy_spec()
    N = 3000
    c = synth.make_cluster(spec, N, 8, seed=44)
    c.hv[:] = 0.0
    c.hv_ts[:] = TS_INVALID
    eng = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts)  # hv NULL
    rng = np.random.default_rng(44)
    idx = rng.choice(N, 25, replace=False).astype(np.int64)
    churn(c, spec, rng, idx, int(synth.NOW0_NS))
    push(eng, c, idx)
    fresh = engine_for(spec, c)
    t0 = int(synth.NOW0_NS)
    assert same_tables(eng.node_steps(t0, t0 + 30 * 10**9), fresh.node_steps(t0, t0 + 30 * 10**9))
    assert np.array_equal(eng.eval(c.now, c.ds)[2], fresh.eval(c.now, c.ds)[2])
    eng.close()
    fresh.close()


def test_update_rejects_bad_indices():
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 100, 1, seed=45)
    eng = engine_for(spec, c)
    val, ts, _ = c.rows(eng.metric_names)
    for idx in ([3, 3], [-1], [100]):
        i = np.array(idx, np.int64)
        with pytest.raises(cd.CraneError):
            eng.update_nodes(i, val[:, :len(i)], ts[:, :len(i)])
        with pytest.raises(cd.CraneError):
            eng.node_steps_subset(0, 10, i)
    eng.update_nodes(np.zeros(0, np.int64), val[:, :0], ts[:, :0])  # k = 0: nothing to do
    eng.close()


def test_state_change_waits_only_for_its_own_streams():
    """quiesce is scoped to the engine's caller streams: engine A's upload_bindings returns
    while engine B still has a long queue of batches in flight on another stream (the
    round-3 form synchronised the device and waited for B too)."""
    import time

    import torch
    spec = cd.default_policy_spec()
    dev = torch.device("cuda", 0)
    cb = synth.make_cluster(spec, 100_000, 10_000, seed=46)
    eb = engine_for(spec, cb)
    sb = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(cb.now).to(dev)
    d_flags = torch.from_numpy(cb.ds).to(dev)
    d_ff = torch.empty((len(cb.now), 100_000), dtype=torch.int8, device=dev)
    d_sc = torch.empty_like(d_ff)
    eb.eval_matrix_async(d_now, d_flags, d_ff, d_sc, stream=sb.cuda_stream)
    sb.synchronize()
    t = time.perf_counter()
    eb.eval_matrix_async(d_now, d_flags, d_ff, d_sc, stream=sb.cuda_stream)
    sb.synchronize()
    one = time.perf_counter() - t
    ca = synth.make_cluster(spec, 2000, 64, n_bindings=20_000, seed=47)
    ea = engine_for(spec, ca)
    sa = torch.cuda.Stream(dev)
    a_now = torch.from_numpy(ca.now).to(dev)
    a_flags = torch.from_numpy(ca.ds).to(dev)
    a_keys = torch.empty(len(ca.now), dtype=torch.int64, device=dev)
    ea.upload_bindings(ca.b_node, ca.b_ts)
    reps = max(8, int(0.4 / max(one, 1e-4)))  # >= 0.4 s of B's batches queued
    for _ in range(reps):
        eb.eval_matrix_async(d_now, d_flags, d_ff, d_sc, stream=sb.cuda_stream)
    now = int(synth.NOW0_NS)
    ea.step_keys_async(now, now, a_now, a_flags, a_keys, sa.cuda_stream)  # A's own async work
    t = time.perf_counter()
    ea.upload_bindings(ca.b_node[::2], ca.b_ts[::2])  # a state change of A: waits for sa only
    waited = time.perf_counter() - t
    b_busy = not sb.query()
    sb.synchronize()
    assert b_busy, f"B's queue ({reps} batches of {one * 1e3:.2f} ms) drained before A's upload returned"
    assert waited < 0.25 * reps * one
    # A's step had finished before its state changed: its keys equal a fresh run's
    ref = torch.empty_like(a_keys)
    ea2 = engine_for(spec, ca)
    ea2.upload_bindings(ca.b_node, ca.b_ts)
    ea2.step_keys_async(now, now, a_now, a_flags, ref, sa.cuda_stream)
    sa.synchronize()
    assert torch.equal(a_keys, ref)
    for e in (ea, ea2, eb):
        e.close()


def test_resize_then_update_equals_fresh_engine_all_time():
    """Nodes joining (crane_dyn_resize_nodes grows the shard: the new rows have no annotations until
    crane_dyn_update_node_steps writes them) and a shrink that drops the last rows: the tables over
    the whole time axis (t0 = INT64_MIN, t1 = INT64_MAX: every expiry fits a row) equal a fresh
    engine holding the final nodes, and the oracle at pod times hours apart."""
    spec = cd.default_policy_spec()
    rng = np.random.default_rng(808)
    c = synth.make_cluster(spec, 3000, 64, seed=808, pod_step_ns=1_800_000_000_000 // 64)
    full = synth.make_cluster(spec, 3500, 64, seed=809)
    keep = 2800  # the engine first holds 2800 nodes, then grows to 3500, then shrinks to 3300
    eng = engine_for(spec)
    val, ts, _ = full.rows(eng.metric_names)
    eng.upload_nodes(val[:, :keep], ts[:, :keep], full.hv[:keep], full.hv_ts[:keep])
    lo, hi = np.iinfo(np.int64).min, np.iinfo(np.int64).max
    eng.resize_nodes(3500)
    tab = list(eng.node_steps(lo, hi))
    # the new rows: no annotations yet (every metric missing: Filter passes, Score from failed terms)
    new = np.arange(keep, 3500)
    rows = eng.update_node_steps(new, val[:, new], ts[:, new], full.hv[new], full.hv_ts[new], lo, hi)
    patch(tab, rows, new)
    churn(full, spec, rng, np.arange(0, 3500, 7), int(synth.NOW0_NS))
    val, ts, _ = full.rows(eng.metric_names)
    idx = np.arange(0, 3500, 7)
    patch(tab, eng.update_node_steps(idx, val[:, idx], ts[:, idx], full.hv[idx], full.hv_ts[idx], lo, hi), idx)
    fresh = engine_for(spec)
    fresh.upload_nodes(val, ts, full.hv, full.hv_ts)
    ref = fresh.node_steps(lo, hi)
    assert same_tables(tab, ref)
    assert same_tables(eng.node_steps(lo, hi), ref)  # (a full rebuild on the grown engine too)
    from oracle import oracle as O
    okm = (ts != TS_INVALID).astype(np.uint8)
    for p in range(0, 64, 9):  # pods half an hour apart: one table answers them all
        now = np.array([c.now[p]], np.int64)
        ff, sc = cd.Engine.table_lookup(tab, now[0])
        off, osc, _ = O.eval_soa(spec, eng.metric_names, okm, val, np.where(okm == 1, ts, 0),
                                 (full.hv_ts != TS_INVALID).astype(np.uint8), full.hv, full.hv_ts, now,
                                 np.zeros(1, np.uint8))
        assert np.array_equal(ff, off[0]) and np.array_equal(sc, osc[0]), p
    eng.resize_nodes(3300)
    assert same_tables(eng.node_steps(lo, hi), [x[:3300] for x in ref])
    fresh.close()
    eng.close()

