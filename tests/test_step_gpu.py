"""Parity of the K3 step path (crane-scheduler_amd/csrc/step.hip) with the oracle.

The step path serves keys-only evaluation (chosen node + chosen score per pod):
K3p partitions pods by DaemonSet flag, K3a folds every node into a step function
of `now` over the batch's time range, K3s evaluates every (pod, node) pair.
These cases aim at its seams: pod times exactly on node expiries (stats.go:42-48
now.Before(ts + dur) is strict), unsorted and duplicated pod times, DaemonSet
mixes that make waves uniform, mixed and all-DaemonSet, segment / tile / chunk
edges (N and P not multiples of 256 / 64 / 1024), and the 8x8 / 16x16 record
shapes.  Reference: plugins.go:39-98 (Filter, Score), utils.go:17-24.
"""
import numpy as np
import pytest

from helpers import engine_for, oracle_soa

pytestmark = pytest.mark.gpu

cd = pytest.importorskip("crane_dyn")
from crane_dyn import synth  # noqa: E402


def _check(spec, c, now, ds):
    off, osc, och = oracle_soa(spec, c, now=now, ds=ds)
    # K3s from the producers' per-tile rows, and searching the records itself; K1's
    # one-step records through its LDS staging, through st.stage always (cap 0), or
    # per block as its counts exceed a small cap; the middle pieces raw or cut into elementary
    # ones (step_pieces 1 always, 0 when it pays, 2 never)
    # the node pass as the streamed step pass (k1_stream 1, the default without dedupe-form K2
    # entries: no record in registers, the stepped records built in LDS in chunks of 64) or the
    # record-holding fused pass (0)
    # (k1_tail: the streamed pass's tail on one wave, 1, or on all four, 4: auto picks by grid size)
    for rows, cap, pc, sf, tl in ((1, 1 << 30, 0, 1, 0), (0, 1 << 30, 0, 1, 0), (1, 0, 1, 1, 0), (0, 6, 0, 1, 0),
                                  (1, 6, 1, 1, 0), (1, 1 << 30, 1, 1, 0), (1, 0, 2, 1, 0), (1, 1 << 30, 0, 0, 0),
                                  (0, 6, 1, 0, 0), (1, 0, 2, 0, 0), (1, 1 << 30, 1, 1, 1), (0, 6, 0, 1, 1),
                                  (1, 0, 2, 1, 1)):
        eng = engine_for(spec, c, opts={"step_rows": rows, "step_lds_cap": cap, "step_pieces": pc, "k1_stream": sf,
                                        "k1_tail": tl})
        _, _, ch, cs = eng.eval(now, ds)
        assert np.array_equal(ch, och), (rows, cap, pc, sf, tl)
        for p in range(len(now)):
            ok = (off[p] < 0) | bool(ds[p])
            assert cs[p] == (osc[p][ok].max() if ok.any() else -1), (rows, cap, pc, sf, tl, p)
        eng.close()


@pytest.mark.parametrize("n_nodes,n_pods,step_ns,ds_frac,seed", [
    (1, 1, 0, 0.0, 1),
    (255, 63, 1_000_000, 0.01, 2),
    (257, 65, 1_000_000_000, 0.5, 3),
    (4099, 1025, 1_000_000, 0.01, 4),
    (3000, 700, 1_700_000_000, 0.05, 5),   # 20-minute batch: almost every node steps
    (20000, 2100, 0, 0.01, 6),             # one `now` for the whole batch: every node flat
    (1000, 300, 60_000_000_000, 1.0, 7),   # all DaemonSet pods
    (6000, 9000, 20_000_000, 0.02, 8),     # 180 s over 9 tiles: middle pieces cut into elementary ones
    (3000, 5000, 200_000_000, 0.3, 9),     # 1000 s: some blocks past the pieces' LDS scratch (raw)
])
def test_step_random_vs_oracle(n_nodes, n_pods, step_ns, ds_frac, seed):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, n_nodes, n_pods, seed=seed, pod_step_ns=step_ns, ds_frac=ds_frac)
    _check(spec, c, c.now, c.ds)


def test_step_pod_times_on_expiries():
    """Pods placed exactly on, and 1 ns either side of, node expiries (ts + period + 5m)."""
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 2000, 1, seed=21)
    rng = np.random.default_rng(3)
    dur = {n: p + 300 * 10**9 for n, p in spec["syncPolicy"]}
    exp = []
    for m, name in enumerate(c.metric_names):
        ok = c.ok[m] == 1
        exp.append(c.ts[m][ok] + dur[name])
    exp.append(c.hv_ts[c.hv_ts != synth.TS_INVALID] + 300 * 10**9)  # hot value: no extra 5m (stats.go:152-166)
    exp = np.concatenate(exp)
    pick = rng.choice(exp, 1500)
    now = np.concatenate([pick, pick - 1, pick + 1]).astype(np.int64)
    rng.shuffle(now)
    ds = (rng.random(len(now)) < 0.02).astype(np.uint8)
    _check(spec, c, now, ds)


def test_step_unsorted_duplicate_times():
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 5000, 1, seed=22)
    rng = np.random.default_rng(4)
    base = synth.NOW0_NS + rng.integers(-600, 600, 300) * 10**9
    now = np.repeat(base, 4).astype(np.int64)
    rng.shuffle(now)
    ds = (rng.random(len(now)) < 0.3).astype(np.uint8)
    _check(spec, c, now, ds)


def test_step_policy_shapes():
    """8x8 and 16x16 records, skipped entries, no priorities, weight sum 0 (NaN/Inf scores)."""
    m = 60 * 10**9
    base = cd.default_policy_spec()
    specs = []
    s = dict(base)
    s["predicate"] = base["predicate"] + [("cpu_usage_max_avg_1d", 0.5), ("mem_usage_max_avg_1d", 0.0),
                                          ("not_synced", 0.1), ("mem_usage_avg_5m", 0.3)]
    specs.append(s)
    s = dict(base)
    s["syncPolicy"] = base["syncPolicy"] + [("m%d" % i, (i + 1) * m) for i in range(10)] + [("zero", 0), ("neg5", -5 * m)]
    s["priority"] = base["priority"] + [("m%d" % i, 0.1 * (i + 1)) for i in range(10)] + [("zero", 1.0), ("neg5", 2.0)]
    s["predicate"] = [("m%d" % i, 0.4 + 0.05 * i) for i in range(10)] + [("neg5", 0.5)]
    specs.append(s)
    s = dict(base)
    s["priority"] = []
    specs.append(s)
    s = dict(base)
    s["priority"] = [("cpu_usage_avg_5m", 1.0), ("mem_usage_avg_5m", -1.0)]
    specs.append(s)
    for i, spec in enumerate(specs):
        c = synth.make_cluster(spec, 777, 90, seed=200 + i, pod_step_ns=20_000_000_000, ds_frac=0.1)
        _check(spec, c, c.now, c.ds)
    # many tiles and a wide batch: the shapes' middle pieces go through step_pieces
    for i, spec in enumerate(specs[:2]):
        c = synth.make_cluster(spec, 1500, 4100, seed=210 + i, pod_step_ns=60_000_000, ds_frac=0.1)
        _check(spec, c, c.now, c.ds)


def test_step_at_large_n():
    """Past one round of resident workgroups (400k nodes): the step path's keys (streamed pass with
    its tail on one wave or on four, the fused pass) equal the per-pair kernel's."""
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 400_000, 1500, seed=30, pod_step_ns=4_000_000, ds_frac=0.02)
    out = []
    for opts in ({"keys_path": 1}, {}, {"k1_tail": 1}, {"k1_tail": 4}, {"k1_stream": 0}):
        eng = engine_for(spec, c, opts=opts)
        _, _, ch, cs = eng.eval(c.now, c.ds)
        out.append((ch, cs))
        eng.close()
    for i in range(1, len(out)):
        assert np.array_equal(out[i][0], out[0][0]) and np.array_equal(out[i][1], out[0][1]), i


def _oracle_hv(spec, c, now_ns):
    from oracle import oracle as O
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, now_ns // 10**9)
    return hv.astype(np.float64), np.full(c.n_nodes, now_ns, np.int64)


def test_step_replayed_batches_with_binding_log():
    """The bench's step (K2 refresh -> keys-only eval) replayed on one stream: K1
    consumes the K2 buckets and zeroes K2's bin cursors in-stream, so every
    replay must give the oracle's choices with hot values from the log."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 20000, 3000, n_bindings=200_000, seed=25, pod_step_ns=3_000_000)
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    now = int(synth.NOW0_NS)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    _, _, och = oracle_soa(spec, c, want_matrix=False, hv_override=_oracle_hv(spec, c, now))
    with torch.cuda.stream(st):
        for rep in range(4):
            eng.refresh_hot_values_async(now, now, st.cuda_stream)
            eng.eval_keys_async(d_now, d_flags, d_keys, st.cuda_stream)
            st.synchronize()
            ch = np.array([cd.key_node(int(k))[0] for k in d_keys.cpu().numpy()])
            assert np.array_equal(ch, och), rep


def test_hot_values_kept_after_consumption():
    """After the node pass has consumed the K2 buckets, a later node pass (records
    made stale by greedy) still sees the refreshed binding-log hot values."""
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 3000, 500, n_bindings=40_000, seed=26, pod_step_ns=0)
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    now = int(c.now[0])
    eng.refresh_hot_values(now, now)
    _, _, ch1, _ = eng.eval(c.now, c.ds)          # consumes the counts
    eng.greedy(50, now, c.ds[:50])                # refreshes at the same now, leaves records stale
    ff, sc, ch2, _ = eng.eval(c.now, c.ds, matrix=True)   # K1 again from the kept hot values (pair kernel)
    off, osc, och = oracle_soa(spec, c, hv_override=_oracle_hv(spec, c, now))
    assert np.array_equal(ch1, och) and np.array_equal(ch2, och)
    assert np.array_equal(ff, off) and np.array_equal(sc, osc)


@pytest.mark.parametrize("delta", [1, 0], ids=["delta", "recount"])
@pytest.mark.parametrize("pods", [5000, 1, 300, 2048])
def test_step_keys_async_matches_oracle(pods, delta):
    """crane_dyn_step_keys_async replayed (K3p riding in K2's launch) at hot-value times that
    move between steps (the delta form adjusts its anchor's counts; recount: the dedupe form):
    each step equals the oracle with binding-log hot values; with kernel timing on
    too (dispatch-stamped events name every kernel of the step)."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 30000, pods, n_bindings=300_000, seed=27, pod_step_ns=2_000_000, ds_frac=0.02)
    eng = engine_for(spec, c, opts={"k2_delta": delta})
    eng.upload_bindings(c.b_node, c.b_ts)
    now = int(synth.NOW0_NS)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    with torch.cuda.stream(st):
        for rep, dt in enumerate((0, 9, -4, 30)):
            t = now + dt * 10**9
            _, _, och = oracle_soa(spec, c, want_matrix=False, hv_override=_oracle_hv(spec, c, t))
            eng.set_profiling(rep == 3)
            eng.step_keys_async(t, t, d_now, d_flags, d_keys, st.cuda_stream)
            st.synchronize()
            ch = np.array([cd.key_node(int(k))[0] for k in d_keys.cpu().numpy()])
            assert np.array_equal(ch, och), rep
    times = eng.stage_times()
    names = [n for n, _ in times]
    want = (["k2_delta+k3p_pods", "k1_stream_steps", "k3s_eval"] if delta else
            ["k2x_dedupe+k3p_pods", "k1_node_pass+k3a_steps", "k3s_eval"])
    assert names == want, names
    assert all(0 < t < 50 for _, t in times), times


@pytest.mark.parametrize("k2", [0, 2, 3], ids=["dedupe", "atomics", "large"])
def test_step_keys_async_k2_forms(k2):
    """The combined step with each K2 form (dedupe: counts consumed by the fused node
    pass from per-block entries; atomics / large: buckets; K3p its own launch) equals the oracle, replayed."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 20000, 3000, n_bindings=400_000, seed=29, pod_step_ns=2_000_000, ds_frac=0.03)
    eng = engine_for(spec, c, opts={"k2_form": k2, "k2_delta": 0})
    eng.upload_bindings(c.b_node, c.b_ts)
    now = int(synth.NOW0_NS)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    _, _, och = oracle_soa(spec, c, want_matrix=False, hv_override=_oracle_hv(spec, c, now))
    with torch.cuda.stream(st):
        for rep in range(3):
            eng.set_profiling(rep == 2)
            eng.step_keys_async(now, now, d_now, d_flags, d_keys, st.cuda_stream)
            st.synchronize()
            ch = np.array([cd.key_node(int(k))[0] for k in d_keys.cpu().numpy()])
            assert np.array_equal(ch, och), rep
    names = [n for n, _ in eng.stage_times()]
    # the dedupe form's per-block entries need the record-holding fused pass; the others stream
    assert ("k1_node_pass+k3a_steps" if k2 == 0 else "k1_stream_steps") in names, names


def test_records_rebuilt_after_keys_step():
    """The fused keys-only step does not write the node records: a matrix eval and a greedy pass after it rebuild them from
    the kept binding-log hot values and still equal the oracle."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 4000, 700, n_bindings=50_000, seed=28, pod_step_ns=3_000_000, ds_frac=0.05)
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    now = int(synth.NOW0_NS)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    off, osc, och = oracle_soa(spec, c, hv_override=_oracle_hv(spec, c, now))
    with torch.cuda.stream(st):
        eng.step_keys_async(now, now, d_now, d_flags, d_keys, st.cuda_stream)
        st.synchronize()
    ch = np.array([cd.key_node(int(k))[0] for k in d_keys.cpu().numpy()])
    assert np.array_equal(ch, och)
    ff, sc, ch2, _ = eng.eval(c.now, c.ds, matrix=True)
    assert np.array_equal(ff, off) and np.array_equal(sc, osc) and np.array_equal(ch2, och)
    _, _, ch3, _ = eng.eval(c.now, c.ds)  # keys-only again, records clean now
    assert np.array_equal(ch3, och)
