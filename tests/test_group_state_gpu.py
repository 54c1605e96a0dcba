"""The group as the real multi-GPU engine (crane_dyn_group_*, group.cpp): its batch slots share one
copy of each shard's inputs, its shard state changes are routed by global node index (the
controller's patches, joining nodes, the BindingRecords heap, the drop-in's answer tables), and its
batch form reduces a window of batches' keys with one collective ordered after the dispatch queues.
Every check compares the group with ONE fresh engine holding the whole cluster in its final state,
and with the CPU oracle on a pod sample.
Reference: pkg/controller/annotator/node.go:88-96,123-146 (patches), binding.go:50-123 (heap),
plugins.go:39-98 + selectHost; cmd/scheduler/main.go:18-32 (one scheduler process)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

cd = pytest.importorskip("crane_dyn")
from crane_dyn import shard, synth  # noqa: E402
from helpers import oracle_soa  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _keys_of(eng, now, pods_now, ds):
    import torch
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    k = torch.empty(len(pods_now), dtype=torch.int64, device=dev)
    eng.step_keys_async(now, now, torch.from_numpy(pods_now).to(dev), torch.from_numpy(ds).to(dev), k, st.cuda_stream)
    st.synchronize()
    return k.cpu().numpy()


def _same_tables(a, b):
    """Answer rows equal where defined: n_steps, the first n_steps breakpoints, n_steps + 1 values
    (the slots past a row's count are not written)."""
    ns_a, bp_a, ff_a, sc_a = a
    ns_b, bp_b, ff_b, sc_b = b
    if not np.array_equal(ns_a, ns_b):
        return False
    j = np.arange(bp_a.shape[1] + 1)[None, :]
    mb = j[:, :-1] < ns_a[:, None]
    mv = j <= ns_a[:, None]
    return (np.array_equal(bp_a[mb], bp_b[mb]) and np.array_equal(ff_a[mv], ff_b[mv])
            and np.array_equal(sc_a[mv], sc_b[mv]))


def test_slots_share_the_shard_inputs():
    """Device memory after the upload does not grow with the group's depth by the shard's SoA and
    binding log: the slots of a shard hold one copy of them (engine.hip ShardData), and only their
    own scratch (the node records) besides."""
    import torch
    spec = cd.default_policy_spec()
    N, B = 20_000, 8_000_000  # the log (96 MB) dwarfs a slot's records (3.2 MB)
    c = synth.make_cluster(spec, N, 16, n_bindings=B, seed=3)
    used = {}
    for depth in (1, 4):
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info(0)[0]
        g = cd.Group(cd.Policy(spec), devices=[0], depth=depth)
        val, ts, _ = c.rows(g.metric_names)
        g.upload_nodes(val, ts, c.hv, c.hv_ts)
        g.upload_bindings(c.b_node, c.b_ts)
        torch.cuda.synchronize()
        used[depth] = free0 - torch.cuda.mem_get_info(0)[0]
        g.close()
    log_bytes = 12 * B
    assert used[1] >= log_bytes // 2, used  # (the measurement sees the log)
    assert used[4] - used[1] < log_bytes // 2, (used, "the slots copied the shard")


@pytest.mark.parametrize("S,depth", [(3, 2), (1, 3)])
def test_group_state_changes_equal_a_fresh_engine(S, depth):
    """S shards on the one GPU (collective 0, the host max-combines), `depth` slots each: patches
    to random global nodes (update_node_steps, rows returned), nodes joining at the end
    (resize_nodes, then their annotations), the controller's binding heap fed with global node
    indices (binding_records, add_bindings with capacity evictions, gc_bindings) — after each, every
    slot's batch keys equal one fresh engine over the whole cluster in its current state, the answer
    tables (node_steps) and hot values are the fresh engine's, and a pod sample equals the oracle."""
    spec = cd.default_policy_spec()
    rng = np.random.default_rng(60 + S)
    N0, P = 12_011, 1_500
    c = synth.make_cluster(spec, N0, P, seed=61 + S, pod_step_ns=5_000_000)
    c2 = synth.make_cluster(spec, N0 + 200, P, seed=71 + S, pod_step_ns=5_000_000)  # patch source
    g = cd.Group(cd.Policy(spec), devices=[0] * S, depth=depth)
    g.set_option("collective", 0)
    names = g.metric_names
    val, ts, _ = c.rows(names)
    val, ts = val.copy(), ts.copy()
    hv, hv_ts = c.hv.copy(), c.hv_ts.copy()
    v2, t2, _ = c2.rows(names)
    g.upload_nodes(val, ts, hv, hv_ts)
    now = int(synth.NOW0_NS)

    def fresh():
        e = cd.Engine(cd.Policy(spec), 0)
        e.upload_nodes(val, ts, hv, hv_ts)
        return e

    def check(e_ref, label, heap=None):
        N = val.shape[1]
        ref = _keys_of(e_ref, now, c.now, c.ds)
        for slot in range(depth + 1):  # every slot (and slot 0 again)
            ch, sc = g.schedule(now, now, c.now, c.ds)
            assert np.array_equal(ch, shard.unpack_keys(ref)[0]), (label, slot)
            assert np.array_equal(sc, shard.unpack_keys(ref)[1]), (label, slot)
        assert _same_tables(g.node_steps(-(2**63), 2**63 - 1), e_ref.node_steps(-(2**63), 2**63 - 1)), label
        if heap is None:
            assert np.array_equal(g.hot_values(), e_ref.hot_values()), label
        # the oracle on a sample: the step refreshes hot values from the log (none: 0) or the heap
        smp = np.unique(np.linspace(0, P - 1, 24).astype(int))
        if heap is None:
            hvo = (np.zeros(N), np.full(N, now, np.int64))
        else:
            _, hvh = O.hot_values(spec, heap[0], heap[1], N, now // 10**9)
            hvo = (hvh.astype(np.float64), np.full(N, now, np.int64))
        cc = synth.make_cluster(spec, 1, 1, seed=1)
        cc.val, cc.ok = val, np.where(ts == synth.TS_INVALID, 0, 1).astype(np.uint8)
        cc.ts, cc.metric_names = ts, list(names)
        _, _, och = oracle_soa(spec, cc, now=c.now[smp], ds=c.ds[smp], want_matrix=False, hv_override=hvo)
        assert np.array_equal(shard.unpack_keys(ref)[0][smp], och), label

    e = fresh()
    e.upload_bindings(np.zeros(0, np.int32), np.zeros(0, np.int64))
    check(e, "upload")
    e.close()
    # the controller's patches: a few hundred nodes across every shard, rows returned
    for rnd in range(2):
        idx = np.unique(rng.integers(0, val.shape[1], 300))
        rows = g.update_node_steps(idx, v2[:, idx], t2[:, idx], c2.hv[idx], c2.hv_ts[idx], -(2**63), 2**63 - 1)
        val[:, idx], ts[:, idx], hv[idx], hv_ts[idx] = v2[:, idx], t2[:, idx], c2.hv[idx], c2.hv_ts[idx]
        e = fresh()
        assert _same_tables(rows, e.node_steps_subset(-(2**63), 2**63 - 1, idx)), rnd
        check(e, f"patch {rnd}")
        e.close()
    # nodes join at the end: the last shard grows, the new rows start without annotations, then
    # the controller's first patch of each
    N1 = val.shape[1] + 37
    g.resize_nodes(N1)
    M = val.shape[0]
    val = np.concatenate([val, np.zeros((M, 37))], 1)
    ts = np.concatenate([ts, np.full((M, 37), synth.TS_INVALID, np.int64)], 1)
    hv = np.concatenate([hv, np.zeros(37)])
    hv_ts = np.concatenate([hv_ts, np.full(37, synth.TS_INVALID, np.int64)])
    assert g.shard(S - 1)[2] == N1
    e = fresh()
    check(e, "grown")
    e.close()
    new = np.arange(N1 - 37, N1)
    src = np.arange(N0, N0 + 37)
    g.update_nodes(new, v2[:, src], t2[:, src], c2.hv[src], c2.hv_ts[src])
    val[:, new], ts[:, new], hv[new], hv_ts[new] = v2[:, src], t2[:, src], c2.hv[src], c2.hv_ts[src]
    e = fresh()
    check(e, "joined")
    e.close()
    # the controller's binding heap, global node indices (evictions: more adds than its size)
    size, gc_tr = 50_000, 300 * 10**9
    g.binding_records(size, gc_tr)
    e = fresh()
    e.binding_records(size, gc_tr)
    nu = now // 10**9
    ops, onode, oarg = [], [], []
    for rnd in range(3):
        bn = rng.integers(-2, N1 + 3, 30_000).astype(np.int32)
        bt = np.sort(rng.integers(nu - 900, nu + 1, 30_000)).astype(np.int64)
        g.add_bindings(bn, bt)
        e.add_bindings(bn, bt)
        ops += [0] * len(bn)
        onode += bn.tolist()
        oarg += bt.tolist()
        if rnd == 1:
            g.gc_bindings(now - 100 * 10**9)
            e.gc_bindings(now - 100 * 10**9)
            ops.append(1)
            onode.append(0)
            oarg.append(nu - 100)
        assert g.binding_count() == e.binding_count(), rnd
    heap = O.binding_heap(size, gc_tr, ops, onode, oarg)  # the controller's heap, restated
    assert g.binding_count() == len(heap[0])
    g.refresh_hot_values(now, now)
    e.refresh_hot_values(now, now)
    assert np.array_equal(g.hot_values(), e.hot_values())
    _, hvh = O.hot_values(spec, heap[0], heap[1], N1, nu)
    assert np.array_equal(g.hot_values(), hvh.astype(np.float64))
    check(e, "heap", heap=heap)
    e.close()
    g.close()


@pytest.mark.parametrize("dispatch,threads", [(-1, 1), (-1, 0), (0, 1)], ids=["queues-workers", "queues-caller",
                                                                             "streams-workers"])
def test_batch_form_one_collective_after_the_queues(dispatch, threads):
    """crane_dyn_group_step_keys_batch with the collective on (a one-rank RCCL communicator on the
    one GPU, "collective" 2): G batches on the slots' dispatch queues (or HIP streams), then ONE
    in-place all-reduce of their keys [G][P] on the group's collective stream, ordered after the
    queues by the flag packet each slot's last batch is followed by (hipStreamWaitValue64).  The
    keys equal a stream engine's per batch; a second window into the other buffer and a third back
    into the first (which waits for the first window's collective) too."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 30_011, 2_000, n_bindings=200_000, seed=81, pod_step_ns=5_000_000)
    c.now, c.ds = synth.make_pods(2_000, seed=82)
    dev = torch.device("cuda", 0)
    G, depth = 6, 4
    g = cd.Group(cd.Policy(spec), devices=[0], depth=depth)
    g.set_option("collective", 2)
    g.set_option("threads", threads)
    g.set_option("dispatch", dispatch)
    val, ts, _ = c.rows(g.metric_names)
    g.upload_nodes(val, ts, c.hv, c.hv_ts)
    g.upload_bindings(c.b_node, c.b_ts)
    span = int(c.now[-1] - c.now[0]) + 1
    eng = cd.Engine(cd.Policy(spec), 0)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    eng.upload_bindings(c.b_node, c.b_ts)
    bufs = [torch.full((G, len(c.now)), -7, dtype=torch.int64, device=dev) for _ in range(2)]
    flags = torch.from_numpy(np.tile(c.ds, (G, 1))).to(dev)
    for w, b in enumerate((0, 1, 0)):
        times = [int(c.now[0]) + (w * G + j) * span for j in range(G)]
        pods = np.stack([c.now + (w * G + j) * span for j in range(G)])
        d_now = torch.from_numpy(pods).to(dev)
        torch.cuda.synchronize()
        g.step_keys_batch(times, times, [d_now], [flags], [bufs[b]])
        if w < 2:
            continue
        g.sync()
        got = bufs[b].cpu().numpy()
        for j in range(G):
            ref = _keys_of(eng, times[j], pods[j], c.ds)
            assert np.array_equal(got[j], ref), (w, j)
    g.sync()
    eng.close()
    g.close()
