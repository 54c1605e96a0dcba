"""Parity of the HIP engine (through the C ABI) with the oracle and the golden vectors.

Bit-exact on filter results (first failing predicate), int64 scores and chosen
nodes, per /root/reference/pkg/plugins/dynamic/{plugins,stats}.go.
"""
import numpy as np
import pytest

from conftest import policy_from_json
from helpers import SH, engine_for, oracle_soa

pytestmark = pytest.mark.gpu

# keys-only evaluations: 0 = the step path (step.hip), 1 = the per-pair kernel (matrix.hip);
# matrix outputs always come from the per-pair kernel
@pytest.fixture(params=[0, 1], ids=["keys_step", "keys_pair"])
def kp(request):
    return {"keys_path": request.param}

cd = pytest.importorskip("crane_dyn")
from crane_dyn import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _eval_annotations(spec, nodes, now, ds):
    eng = engine_for(spec)
    val, ts, hv, hv_ts = cd.parse_nodes(eng.metric_names, nodes, SH)
    eng.upload_nodes(val, ts, hv, hv_ts)
    return eng.eval(np.asarray(now, np.int64), np.asarray(ds, np.uint8), matrix=True)


def test_kats(kats):
    for k in kats["kats"]:
        spec = policy_from_json(k["policy"])
        ff, sc, ch, cs = _eval_annotations(spec, [k["annotations"]], [k["now_ns"]], [k["daemonset"]])
        assert ff[0, 0] == k["expect_filter"], k["name"]
        assert sc[0, 0] == k["expect_score"], k["name"]
        assert ch[0] == (0 if k["expect_filter"] < 0 else -1), k["name"]
        assert cs[0] == (k["expect_score"] if k["expect_filter"] < 0 else -1), k["name"]


def test_golden_cluster(cluster_small):
    c = cluster_small
    spec = policy_from_json(c["policy"])
    now = [p["now_ns"] for p in c["pods"]]
    ds = [p["daemonset"] for p in c["pods"]]
    ff, sc, ch, _ = _eval_annotations(spec, c["nodes"], now, ds)
    assert ff.tolist() == c["expect_filter"]
    assert sc.tolist() == c["expect_score"]
    assert ch.tolist() == c["expect_chosen"]


@pytest.mark.parametrize("n_nodes,n_pods,seed", [(1, 1, 1), (100, 1, 2), (257, 33, 3), (5000, 64, 4), (3000, 700, 5)])
def test_random_vs_oracle(n_nodes, n_pods, seed, kp):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, n_nodes, n_pods, seed=seed, pod_step_ns=1_700_000_000)
    eng = engine_for(spec, c, opts=kp)
    ff, sc, ch, cs = eng.eval(c.now, c.ds, matrix=True)
    off, osc, och = oracle_soa(spec, c)
    assert np.array_equal(ff, off)
    assert np.array_equal(sc, osc)
    assert np.array_equal(ch, och)
    _, _, ch2, cs2 = eng.eval(c.now, c.ds)  # keys only
    assert np.array_equal(ch2, och) and np.array_equal(cs2, cs)
    # chosen score equals the max feasible score
    for p in range(n_pods):
        feas = (off[p] < 0)
        assert cs[p] == (osc[p][feas].max() if feas.any() else -1)


def test_keys_only_matches_matrix(kp):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 20000, 300, seed=11, pod_step_ns=3_000_000_000)
    eng = engine_for(spec, c, opts=kp)
    _, _, ch_m, cs_m = eng.eval(c.now, c.ds, matrix=True)
    _, _, ch, cs = eng.eval(c.now, c.ds, matrix=False)
    assert np.array_equal(ch, ch_m) and np.array_equal(cs, cs_m)
    _, _, och = oracle_soa(spec, c, want_matrix=False)
    assert np.array_equal(ch, och)


def test_no_hot_value_and_empty_shard():
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 50, 4, seed=7)
    eng = cd.Engine(cd.Policy(spec))
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts)  # no node_hot_value annotations at all
    ff, sc, ch, _ = eng.eval(c.now, c.ds, matrix=True)
    off, osc, och = O.eval_soa(spec, c.metric_names, c.ok, c.val, np.where(c.ok == 1, c.ts, 0),
                               np.zeros(50, np.uint8), np.zeros(50), np.zeros(50, np.int64), c.now, c.ds)
    assert np.array_equal(ff, off) and np.array_equal(sc, osc) and np.array_equal(ch, och)
    M = len(eng.metric_names)
    eng.upload_nodes(np.zeros((M, 0)), np.zeros((M, 0), np.int64))
    _, _, ch, cs = eng.eval(c.now, c.ds)
    assert (ch == -1).all() and (cs == -1).all()


def test_policy_variants(kp):
    """Non-default policy shapes exercise the 8x8 and 16x16 NodeRec kernels and skipped entries."""
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
    s["priority"] = [("cpu_usage_avg_5m", 1.0), ("mem_usage_avg_5m", -1.0)]  # weight sum 0 -> NaN/Inf scores
    specs.append(s)
    for i, spec in enumerate(specs):
        c = synth.make_cluster(spec, 777, 40, seed=100 + i, pod_step_ns=20_000_000_000)
        eng = engine_for(spec, c, opts=kp)
        ff, sc, ch, _ = eng.eval(c.now, c.ds, matrix=True)
        off, osc, och = oracle_soa(spec, c)
        assert np.array_equal(ff, off), i
        assert np.array_equal(sc, osc), i
        assert np.array_equal(ch, och), i
        assert np.array_equal(eng.eval(c.now, c.ds)[2], och), i


def test_hot_values_vs_oracle(kats):
    """KAT-11 through the engine: every metric fresh at 0.0 (base score 100), so score = 100 - 10*hv."""
    h = kats["hot"]["KAT-11"]
    spec = policy_from_json(h["policy"])
    b = np.array(h["bindings"], np.int64)
    eng = cd.Engine(cd.Policy(spec))
    M, N = len(eng.metric_names), h["n_nodes"]
    now_ns = h["now_unix"] * 10**9
    eng.upload_nodes(np.zeros((M, N)), np.full((M, N), now_ns, np.int64))
    eng.upload_bindings(b[:, 0], b[:, 1])
    eng.refresh_hot_values(now_ns, now_ns)
    _, sc, _, _ = eng.eval(np.array([now_ns]), matrix=True)
    assert sc[0].tolist() == [max(0, 100 - 10 * v) for v in h["expect_hv"]]
    assert sc[0, 0] == 50  # hv = 5 (SURVEY KAT-11)


@pytest.mark.parametrize("k2", [0, 2, 3], ids=["dedupe", "atomics", "large"])
@pytest.mark.parametrize("n_nodes,n_bind,seed", [(1000, 50_000, 1), (20_000, 300_000, 2), (100, 10, 3),
                                                 (70_000, 2_000_000, 4), (40_000, 5_000_000, 5)])
def test_hot_values_random(n_nodes, n_bind, seed, k2):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, n_nodes, 16, n_bindings=n_bind, seed=seed, pod_step_ns=10_000_000_000)
    # include bindings for nodes outside the shard
    bn = c.b_node.copy()
    bn[::97] = -1
    bn[1::101] = n_nodes + 5
    eng = engine_for(spec, c, opts={"k2_form": k2, "k2_delta": 0})
    eng.upload_bindings(bn, c.b_ts)
    now = int(c.now[0])
    eng.refresh_hot_values(now, now)
    _, cnt_hv = O.hot_values(spec, bn, c.b_ts, n_nodes, now // 10**9)
    ff, sc, ch, _ = eng.eval(c.now, c.ds, matrix=True)
    off, osc, och = oracle_soa(spec, c, hv_override=(cnt_hv.astype(np.float64), np.full(n_nodes, now, np.int64)))
    assert np.array_equal(ff, off) and np.array_equal(sc, osc) and np.array_equal(ch, och)


@pytest.mark.parametrize("k2", [0, 3, "delta"], ids=["dedupe", "large", "delta"])
@pytest.mark.parametrize("order", ["sorted", "ties", "shuffled", "sorted_off", "all_old", "all_new", "one_out"])
def test_hot_values_time_ordered_log(order, k2):
    """A time-ordered log (a ring appended as bindings happen): K2 reads only the widest
    window's suffix and ranks each binding by its position (engine option k2_sorted, checked
    at upload).  Equal to the oracle's per-binding timestamp test (binding.go:85-91) with runs
    of equal stamps on the cutoffs, a shuffled log (the timestamp path), the option off, every
    binding older than the widest window, every binding inside the narrowest, one just out."""
    spec = cd.default_policy_spec()
    n_nodes, n_bind = 30_000, 400_000
    c = synth.make_cluster(spec, n_nodes, 32, n_bindings=n_bind, seed=51, pod_step_ns=3_000_000_000)
    now = int(c.now[0])
    nu = now // 10**9
    bn, bt = c.b_node.copy(), c.b_ts.copy()
    bn[::89] = -1
    bn[5::97] = n_nodes + 1
    if order == "ties":  # stamps exactly on the cutoffs (now - 300 s, now - 60 s) and one second around
        edge = np.array([nu - 301, nu - 300, nu - 299, nu - 61, nu - 60, nu - 59], np.int64)
        bt = np.sort(np.concatenate([bt[: n_bind - 6 * (n_bind // 12)], np.repeat(edge, n_bind // 12)]))
    if order == "all_old":
        bt = np.sort(bt) - 10_000
    if order == "all_new":
        bt = np.full(n_bind, nu, np.int64)
    if order == "one_out":
        bt = np.full(n_bind, nu, np.int64)
        bt[0] = nu - 300  # not > cutoff: outside every window
    opts = {} if k2 == "delta" else {"k2_form": k2, "k2_delta": 0}
    if order == "sorted_off":
        opts["k2_sorted"] = 0
    if order == "shuffled":
        p = np.random.default_rng(51).permutation(n_bind)
        bn, bt = bn[p], bt[p]
    eng = engine_for(spec, c, opts=opts)
    eng.upload_bindings(bn, bt)
    for rep in range(2):
        eng.refresh_hot_values(now + rep * 7 * 10**9, now)
        _, cnt_hv = O.hot_values(spec, bn, bt, n_nodes, nu + rep * 7)
        assert np.array_equal(eng.hot_values(), cnt_hv.astype(np.float64)), rep
    eng.refresh_hot_values(now, now)
    _, cnt_hv = O.hot_values(spec, bn, bt, n_nodes, nu)
    _, _, ch, _ = eng.eval(c.now, c.ds)
    _, _, och = oracle_soa(spec, c, want_matrix=False, hv_override=(cnt_hv.astype(np.float64),
                                                                    np.full(n_nodes, now, np.int64)))
    assert np.array_equal(ch, och)
    eng.close()


def test_hot_values_delta_sequence():
    """Delta form (engine option k2_delta): after an anchor refresh, a time-ordered log's refresh
    reads only the bindings whose window rank changed (between the anchor's and this refresh's
    suffix starts) and adjusts the anchor's counts.  Each refresh of a sequence of times --
    forward, back past the anchor, within one second, a jump past half the suffix (re-anchor),
    two refreshes with no read between (the first's adjustments dropped), a new log and a
    resized node set (anchor dropped) -- equals the oracle (binding.go:85-91)."""
    spec = cd.default_policy_spec()
    n_nodes, n_bind = 30_000, 400_000
    c = synth.make_cluster(spec, n_nodes, 32, n_bindings=n_bind, seed=53, pod_step_ns=3_000_000_000)
    now = int(c.now[0])
    nu = now // 10**9
    bn, bt = c.b_node.copy(), c.b_ts.copy()
    bn[::89] = -1
    bn[5::97] = n_nodes + 1
    eng = engine_for(spec, c)
    eng.upload_bindings(bn, bt)

    def check(dt, nn=n_nodes, b=(bn, bt), read=True):
        eng.refresh_hot_values(now + dt * 10**9, now)
        if read:
            _, cnt_hv = O.hot_values(spec, b[0], b[1], nn, nu + dt)
            assert np.array_equal(eng.hot_values(), cnt_hv.astype(np.float64)), dt

    for dt in (0, 7, 13, 13, -25, -24, 0, 40, -290, -200, 30):
        check(dt)
    check(-100, read=False)
    check(-90, read=False)
    check(5)
    # a new log: the anchor goes
    bt2 = np.sort(bt + np.random.default_rng(3).integers(-30, 30, n_bind))
    eng.upload_bindings(bn, bt2)
    for dt in (5, 11, -9):
        check(dt, b=(bn, bt2))
    # fewer nodes: bindings to the dropped ones fall out
    eng.resize_nodes(n_nodes - 1000)
    for dt in (-9, 2):
        check(dt, nn=n_nodes - 1000, b=(bn, bt2))
    eng.close()


@pytest.mark.parametrize("k2", [0, 3, 2], ids=["dedupe", "large", "atomics"])
@pytest.mark.parametrize("case", ["one_hot_node", "eight_windows", "last_node", "odd_counts"])
def test_hot_values_dedupe_edges(case, k2):
    """Dedupe-form K2 (per-workgroup (node, bucket) aggregation, counts read by the
    node pass) at its packing limits: a region whose 2048 bindings all hit one node
    (count field), eight windows (bucket field), the shard's last node and bindings
    past the shard; the large form's and the atomics form's the same.  odd_counts: hotValue.count negative
    and past 32 bits (the node pass divides in u32 only when both operands fit;
    Go's int64 division truncates toward zero otherwise, node.go:117)."""
    m = 60 * 10**9
    spec = cd.default_policy_spec()
    n_nodes, n_bind = 5000, 200_000
    if case == "eight_windows":
        spec["hotValue"] = [(k * 40 * 10**9, c) for k, c in zip(range(1, 9), [1, 2, 3, 5, 7, 11, 13, 1])]
    if case == "odd_counts":
        spec["hotValue"] = [(5 * m, -3), (1 * m, 2**32 + 1), (3 * m, 7)]
    c = synth.make_cluster(spec, n_nodes, 64, n_bindings=n_bind, seed=31, pod_step_ns=5_000_000_000)
    bn = c.b_node.copy()
    if case in ("one_hot_node", "odd_counts"):
        bn[: 3 * 2048 + 5] = 4321  # whole source regions on one node
        bn[-4096:] = 17
    if case == "last_node":
        bn[::3] = n_nodes - 1
        bn[1::7] = n_nodes  # past the shard: ignored
        bn[2::11] = -3
    opts = {"k2_form": k2, "k2_delta": 0}
    eng = engine_for(spec, c, opts=opts)
    eng.upload_bindings(bn, c.b_ts)
    now = int(c.now[0])
    for rep in range(2):  # a second refresh after the first was consumed
        eng.refresh_hot_values(now, now)
        _, cnt_hv = O.hot_values(spec, bn, c.b_ts, n_nodes, now // 10**9)
        ff, sc, ch, _ = eng.eval(c.now, c.ds, matrix=True)
        off, osc, och = oracle_soa(spec, c, hv_override=(cnt_hv.astype(np.float64),
                                                         np.full(n_nodes, now, np.int64)))
        assert np.array_equal(ff, off) and np.array_equal(sc, osc) and np.array_equal(ch, och), rep
    eng.refresh_hot_values(now, now)  # read back before any node pass consumed it
    assert np.array_equal(eng.hot_values(), cnt_hv.astype(np.float64))


@pytest.mark.slow
def test_hot_values_large_form_16m():
    """The cold-leg size (4M nodes x 16M bindings), where the dedupe form's count/offset
    matrix passes its cap and the large form runs by default: hot values equal the oracle's
    (binding.go:81-97, node.go:113-121) and the atomics form's, before and after a K1 pass
    consumed them; a pod sample's Filter/Score/argmax equals the oracle over all 4M nodes."""
    spec = cd.default_policy_spec()
    N, B = 4_000_000, 16_000_000
    c = synth.make_cluster(spec, N, 8, n_bindings=B, seed=7, pod_step_ns=20_000_000_000)
    bn = c.b_node.copy()
    bn[::1009] = -1
    bn[1::1013] = N + 3
    eng = engine_for(spec, c)
    eng.upload_bindings(bn, c.b_ts)
    now = int(synth.NOW0_NS)
    _, cnt_hv = O.hot_values(spec, bn, c.b_ts, N, now // 10**9)
    ref = cnt_hv.astype(np.float64)
    eng.set_profiling(True)
    eng.refresh_hot_values(now, now)
    assert [n for n, _ in eng.stage_times()] == ["k2l_partition", "k2y_bin_hist"]
    eng.set_profiling(False)
    assert np.array_equal(eng.hot_values(), ref)
    _, _, ch, _ = eng.eval(c.now, c.ds)
    _, _, och = oracle_soa(spec, c, want_matrix=False, hv_override=(ref, np.full(N, now, np.int64)))
    assert np.array_equal(ch, och)
    eng.refresh_hot_values(now, now)  # again: the buckets are rewritten whole, nothing left to zero
    assert np.array_equal(eng.hot_values(), ref)
    for srt in (0, 1):  # the ordered and the stamp path
        eng.set_option("k2_sorted", srt)
        eng.refresh_hot_values(now, now)
        assert np.array_equal(eng.hot_values(), ref), srt
    eng.set_option("k2_form", 2)
    eng.refresh_hot_values(now, now)
    assert np.array_equal(eng.hot_values(), ref)
    eng.set_option("k2_form", 0)
    eng.refresh_hot_values(now, now)
    assert np.array_equal(eng.hot_values(), ref)


def test_division_exactness_sweep(kp):
    """Dense random usages: int(score/weight) must match the CPU bit for bit (KAT-3/4 FMA traps)."""
    spec = cd.default_policy_spec()
    rng = np.random.default_rng(5)
    N = 200_000
    c = synth.make_cluster(spec, N, 1, seed=9, invalid=False)
    r = rng.random(c.val.shape)
    dec = rng.integers(1, 4, c.val.shape)
    c.val = np.select([dec == 1, dec == 2], [np.round(r, 1), np.round(r, 2)], np.round(r, 3))  # 1-3 decimals
    c.ts[:] = synth.NOW0_NS
    c.hv_ts[:] = synth.TS_INVALID
    eng = engine_for(spec, c, opts=kp)
    _, sc, _, _ = eng.eval(c.now, c.ds, matrix=True)
    off, osc, och = oracle_soa(spec, c)
    assert np.array_equal(sc, osc)
    _, _, ch, cs = eng.eval(c.now, c.ds)
    assert ch[0] == och[0] and cs[0] == osc[0][(off[0] < 0) | bool(c.ds[0])].max()


def test_quotient_adversarial(kp):
    """Two-priority policies whose score/weight lands exactly on, and one ulp around, integers."""
    m = 60 * 10**9
    rng = np.random.default_rng(17)
    for w in (0.3, 1.7, 2.0, 0.1, 3.0):
        spec = {"syncPolicy": [("a", 3 * m), ("b", 3 * m)], "predicate": [],
                "priority": [("a", w), ("b", w / 3.0)], "hotValue": [(5 * m, 5)]}
        N = 4096
        c = synth.make_cluster(spec, N, 1, seed=int(w * 100), invalid=False)
        # usages u with (1-u)*w*100 near integer multiples of the weight sum
        k = rng.integers(0, 140, N)
        base = 1.0 - k / 100.0
        ulps = rng.integers(-3, 4, N)
        u = np.array([np.nextafter(b, np.inf if d > 0 else -np.inf) if d else b for b, d in zip(base, ulps)])
        for _ in range(2):
            u = np.where(ulps > 1, np.nextafter(u, np.inf), np.where(ulps < -1, np.nextafter(u, -np.inf), u))
        c.val[0] = np.abs(u)
        c.val[1] = np.abs(rng.choice([0.0, 0.5, 1.0, 1.5], N))
        c.ts[:] = synth.NOW0_NS
        c.hv_ts[:] = synth.TS_INVALID
        eng = engine_for(spec, c, opts=kp)
        _, sc, _, _ = eng.eval(c.now, c.ds, matrix=True)
        _, osc, och = oracle_soa(spec, c)
        assert np.array_equal(sc, osc), w
        assert np.array_equal(eng.eval(c.now, c.ds)[2], och), w


def test_config2_full_matrix():
    """BASELINE config 2 exactly (5,000 nodes x 1,000 pods, default policy, no binding
    log): the full first-fail and score matrices and every chosen node against the
    oracle bit for bit, through the host API (int64 and compact int8 scores), the
    device-resident matrix form, and the keys-only step path."""
    import torch
    cfg = synth.CONFIGS[2]
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, cfg["nodes"], cfg["pods"], seed=20250215 + 2)
    eng = engine_for(spec, c)
    off, osc, och = oracle_soa(spec, c)
    ff, sc, ch, cs = eng.eval(c.now, c.ds, matrix=True)
    assert np.array_equal(ff, off) and np.array_equal(sc, osc) and np.array_equal(ch, och)
    ff8, sc8, ch8, cs8 = eng.eval(c.now, c.ds, matrix=True, compact=True)
    assert np.array_equal(ff8, off) and np.array_equal(sc8.astype(np.int64), osc)
    assert np.array_equal(ch8, och) and np.array_equal(cs8, cs)
    _, _, chk, csk = eng.eval(c.now, c.ds)  # keys-only: the step path
    assert np.array_equal(chk, och) and np.array_equal(csk, cs)
    dev = torch.device("cuda", 0)
    P, N = cfg["pods"], cfg["nodes"]
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    ld = N + 64  # padded rows
    d_ff = torch.full((P, ld), 77, dtype=torch.int8, device=dev)
    d_sc = torch.full((P, ld), 77, dtype=torch.int8, device=dev)
    d_keys = torch.empty(P, dtype=torch.int64, device=dev)
    eng.eval_matrix_async(d_now, d_flags, d_ff, d_sc, d_keys, ld=ld)
    torch.cuda.synchronize()
    assert np.array_equal(d_ff[:, :N].cpu().numpy(), off) and np.array_equal(d_sc[:, :N].cpu().numpy(), osc)
    assert (d_ff[:, N:] == 77).all() and (d_sc[:, N:] == 77).all()  # padding untouched
    from crane_dyn.shard import unpack_keys
    node, score = unpack_keys(d_keys.cpu().numpy())
    assert np.array_equal(node, och) and np.array_equal(score, cs)


@pytest.mark.slow
def test_config3_full_size_parity():
    """BASELINE config 3 (100k nodes x 10k pods, hot values from a 1M-entry binding log):
    every pod's chosen node from the device-resident key path; a 96-pod sample
    checked against the oracle bit for bit, and size-independent properties on all pods."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 100_000, 10_000, n_bindings=1_000_000, seed=20253215)
    eng = engine_for(spec, c)
    eng.upload_bindings(c.b_node, c.b_ts)
    now_sync = int(synth.NOW0_NS)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    with torch.cuda.stream(st):
        eng.refresh_hot_values_async(now_sync, now_sync, st.cuda_stream)
        eng.node_pass_async(st.cuda_stream)
        eng.eval_keys_async(d_now, d_flags, d_keys, st.cuda_stream)
    st.synchronize()
    keys = d_keys.cpu().numpy()
    node = np.where(keys < 0, -1, 0xFFFFFFFF - (keys & 0xFFFFFFFF))
    score = np.where(keys < 0, -1, keys >> 32)
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, now_sync // 10**9)
    hv_over = (hv.astype(np.float64), np.full(c.n_nodes, now_sync, np.int64))
    sample = np.unique(np.concatenate([np.arange(32), np.linspace(0, 9999, 48).astype(int), np.flatnonzero(c.ds)[:16]]))
    off, osc, och = oracle_soa(spec, c, now=c.now[sample], ds=c.ds[sample], hv_override=hv_over)
    assert np.array_equal(node[sample], och)
    for i, p in enumerate(sample):
        feas = (off[i] < 0)
        assert score[p] == (osc[i][feas].max() if feas.any() else -1)
    # properties on all pods: scores in range; later pods never see more fresh metrics
    assert ((score >= 0) & (score <= 100)).all()
    # host-API path agrees with the device-resident path on a slice
    _, _, ch, cs = eng.eval(c.now[:512], c.ds[:512])
    assert np.array_equal(ch, node[:512]) and np.array_equal(cs, score[:512])


def test_hot_values_readback_matches_controller():
    """crane_dyn_hot_values after a refresh = the controller's annotateNodeHotValue
    (node.go:113-121) over the binding log, per node; before any refresh it is the
    uploaded annotation value."""
    from oracle import oracle as O
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 5000, 1, n_bindings=200_000, seed=31)
    eng = engine_for(spec, c)
    assert np.array_equal(eng.hot_values(), c.hv)
    eng.upload_bindings(c.b_node, c.b_ts)
    now = int(synth.NOW0_NS)
    eng.refresh_hot_values(now, now)
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, now // 10**9)
    assert np.array_equal(eng.hot_values(), hv.astype(np.float64))
    _ = eng.eval(c.now[:1], c.ds[:1])  # consumed by the node pass: still the same values
    assert np.array_equal(eng.hot_values(), hv.astype(np.float64))


def test_config4_shard_parity():
    """BASELINE config 4, one rank's shard (125k nodes, node_offset 3 x 125k) x 100k pods
    spread over 100 s: the step tables carry many one- and multi-step nodes and K3s
    stages them over several rounds; a 160-pod sample (incl. DaemonSet pods) is
    checked against the oracle bit for bit, global indices include the offset."""
    import torch
    spec = cd.default_policy_spec()
    N, P, off = 125_000, 100_000, 3 * 125_000
    c = synth.make_cluster(spec, N, P, n_bindings=1_000_000, seed=20254215)
    eng = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts, node_offset=off)
    eng.upload_bindings(c.b_node, c.b_ts)
    now_sync = int(synth.NOW0_NS)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(P, dtype=torch.int64, device=dev)
    with torch.cuda.stream(st):
        eng.step_keys_async(now_sync, now_sync, d_now, d_flags, d_keys, st.cuda_stream)
    st.synchronize()
    keys = d_keys.cpu().numpy()
    node = np.where(keys < 0, -1, 0xFFFFFFFF - (keys & 0xFFFFFFFF))
    score = np.where(keys < 0, -1, keys >> 32)
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, N, now_sync // 10**9)
    hv_over = (hv.astype(np.float64), np.full(N, now_sync, np.int64))
    sample = np.unique(np.concatenate([np.arange(16), np.linspace(0, P - 1, 128).astype(int),
                                       np.flatnonzero(c.ds)[::max(1, int(c.ds.sum()) // 16)][:16]]))
    offm, osc, och = oracle_soa(spec, c, now=c.now[sample], ds=c.ds[sample], hv_override=hv_over)
    assert np.array_equal(node[sample], np.where(och < 0, -1, och + off))
    for i, p in enumerate(sample):
        feas = (offm[i] < 0) | bool(c.ds[p])
        assert score[p] == (osc[i][feas].max() if feas.any() else -1)
    assert ((score >= 0) & (score <= 100)).all()


@pytest.mark.parametrize("N,horizon_s,seed", [(3000, 60, 71), (20_000, 600, 72), (5, 3600, 73)])
def test_node_steps_tables(N, horizon_s, seed):
    """crane_dyn_node_steps (the drop-in plugin's answer tables): at pod times across the
    horizon — on breakpoints, one ns either side, both ends — the looked-up first-fail and
    score equal the oracle's per-call answers for every node (plugins.go:39-98)."""
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, N, 4, seed=seed)
    eng = engine_for(spec, c)
    t0 = int(synth.NOW0_NS) - 7 * 10**9
    t1 = t0 + horizon_s * 10**9
    tab = eng.node_steps(t0, t1)
    ns, bp = tab[0], tab[1]
    assert (ns <= bp.shape[1]).all()
    bps = np.unique(np.concatenate([bp[i, :ns[i]] for i in range(N)] + [np.array([t0], np.int64)]))
    rng = np.random.default_rng(seed)
    pick = rng.choice(bps, min(12, len(bps)), replace=False)
    times = np.unique(np.concatenate([pick, pick - 1, pick + 1, [t0, t1 - 1]]))
    times = times[(times >= t0) & (times < t1)]
    off, osc, _ = oracle_soa(spec, c, now=times.astype(np.int64), ds=np.zeros(len(times), np.uint8))
    for k, t in enumerate(times):
        ff, sc = cd.Engine.table_lookup(tab, int(t))
        assert np.array_equal(ff, off[k]) and np.array_equal(sc, osc[k]), int(t)
    eng.close()
