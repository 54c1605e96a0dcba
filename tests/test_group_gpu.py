"""The node-shard group through the C ABI (crane_dyn_group_*, group.cpp): one process driving the
shard engines of several devices, their keys max-combined by an in-library RCCL all-reduce
(ncclCommInitAll + ncclAllReduce(int64, ncclMax)).  On the one-GPU box: a one-rank communicator
(option "collective" 2) from worker threads and from the caller's thread inside
ncclGroupStart/End, and several shards on the one device combined on the host ("collective" 0),
each against a single engine over the whole cluster and the CPU oracle.
Reference: SURVEY 8(b) crane_dyn_create(..., device_count, ...); cmd/scheduler/main.go:18-32 (one
scheduler process); plugins.go:39-98 + upstream selectHost; binding.go:81-97."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

cd = pytest.importorskip("crane_dyn")
from crane_dyn import shard, synth  # noqa: E402
from conftest import ROOT  # noqa: E402
from helpers import oracle_soa  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _tied_cluster(n_nodes, n_pods, seed, n_bind):
    """Equal-score copies of node 3 in later shards: the combine must pick the lowest global index."""
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, n_nodes, n_pods, n_bindings=n_bind, seed=seed, pod_step_ns=3_000_000)
    for dst in (n_nodes // 2 + 1, n_nodes - 5):
        c.val[:, dst], c.ts[:, dst], c.ok[:, dst] = c.val[:, 3], c.ts[:, 3], c.ok[:, 3]
        c.hv[dst], c.hv_ts[dst] = c.hv[3], c.hv_ts[3]
    for n in (3, n_nodes // 2 + 1, n_nodes - 5):
        c.val[:, n], c.ok[:, n], c.ts[:, n] = 0.0, 1, synth.NOW0_NS
        c.hv[n], c.hv_ts[n] = 0.0, synth.NOW0_NS
    # the copies bound alike: equal hot values from the log too
    return spec, c


def _reference(spec, c, now):
    """One engine over the whole cluster (its keys) and the oracle's chosen nodes."""
    import torch
    dev = torch.device("cuda", 0)
    eng = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    eng.upload_bindings(c.b_node, c.b_ts)
    st = torch.cuda.Stream(dev)
    k = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    eng.step_keys_async(now, now, torch.from_numpy(c.now).to(dev), torch.from_numpy(c.ds).to(dev), k, st.cuda_stream)
    st.synchronize()
    eng.close()
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, now // 10**9)
    _, _, och = oracle_soa(spec, c, want_matrix=False,
                           hv_override=(hv.astype(np.float64), np.full(c.n_nodes, now, np.int64)))
    return k.cpu().numpy(), och, val, ts


@pytest.mark.parametrize("threads", [1, 0], ids=["workers", "caller-thread"])
def test_group_one_rank_rccl_equals_engine_and_oracle(threads):
    """n_dev = 1 with the RCCL communicator forced on (a one-rank all-reduce after every batch):
    the async form over two batch slots, replayed, and the host-array schedule equal one engine
    and the oracle."""
    import torch
    spec, c = _tied_cluster(20_011, 2_100, 4242, 200_000)
    now = int(synth.NOW0_NS)
    ref_keys, och, val, ts = _reference(spec, c, now)
    assert np.array_equal(shard.unpack_keys(ref_keys)[0], och)
    g = cd.Group(cd.Policy(spec), devices=[0], depth=2)
    g.set_option("collective", 2)
    g.set_option("threads", threads)
    g.upload_nodes(val, ts, c.hv, c.hv_ts)
    g.upload_bindings(c.b_node, c.b_ts)
    assert g.shard(0) == (0, 0, c.n_nodes)
    dev = torch.device("cuda", 0)
    d_now, d_flags = torch.from_numpy(c.now).to(dev), torch.from_numpy(c.ds).to(dev)
    keys = [torch.empty(len(c.now), dtype=torch.int64, device=dev) for _ in range(2)]
    fns = [g.step_keys_fn([d_now], [d_flags], [keys[s]]) for s in range(2)]
    for b in range(6):  # batch b on slot b % 2, key buffer b % 2 (ordered by the slot's stream)
        fns[b % 2](now, now)
    g.sync()
    for s in range(2):
        assert np.array_equal(keys[s].cpu().numpy(), ref_keys), s
    ch, sc = g.schedule(now, now, c.now, c.ds)
    assert np.array_equal(ch, och)
    assert np.array_equal(sc, shard.unpack_keys(ref_keys)[1])
    g.close()


@pytest.mark.parametrize("S,threads", [(3, 1), (8, 1), (4, 0)])
def test_group_shards_on_one_device_host_combine(S, threads):
    """S shards of one cluster on the one GPU (the device listed S times), each with its own nodes'
    bindings, combined on the host ("collective" 0): equal to one engine and the oracle, with
    equal-score ties across shard boundaries going to the lowest global index; the async form
    leaves each shard's keys, whose max is the same."""
    import torch
    spec, c = _tied_cluster(30_011, 3_000, 777 + S, 300_000)
    now = int(synth.NOW0_NS)
    ref_keys, och, val, ts = _reference(spec, c, now)
    g = cd.Group(cd.Policy(spec), devices=[0] * S, depth=1)
    g.set_option("collective", 0)
    g.set_option("threads", threads)
    g.upload_nodes(val, ts, c.hv, c.hv_ts)
    g.upload_bindings(c.b_node, c.b_ts)
    for i in range(S):
        assert g.shard(i) == (0, *shard.shard_range(c.n_nodes, S, i))
    ch, sc = g.schedule(now, now, c.now, c.ds)
    assert np.array_equal(ch, och)
    assert (ch == 3).sum() > 0 and not np.isin(ch, [c.n_nodes // 2 + 1, c.n_nodes - 5]).any()
    dev = torch.device("cuda", 0)
    d_now, d_flags = torch.from_numpy(c.now).to(dev), torch.from_numpy(c.ds).to(dev)
    keys = [torch.empty(len(c.now), dtype=torch.int64, device=dev) for _ in range(S)]
    g.step_keys_async(now, now, [d_now] * S, [d_flags] * S, keys)
    g.sync()
    assert np.array_equal(torch.stack(keys).max(0).values.cpu().numpy(), ref_keys)
    g.close()


def test_group_errors_and_empty_shards():
    """Argument and state errors come back as CraneError with the group's message; more shards
    than nodes leave empty shards that contribute no node; the collective refuses a repeated
    device."""
    spec = cd.default_policy_spec()
    pol = cd.Policy(spec)
    with pytest.raises(cd.CraneError, match="not visible"):
        cd.Group(pol, devices=[9999])
    g = cd.Group(pol, devices=[0, 0, 0, 0])
    with pytest.raises(cd.CraneError, match="upload nodes"):
        g.schedule(0, 0, np.zeros(4, np.int64))
    c = synth.make_cluster(spec, 3, 40, seed=5, pod_step_ns=1_000_000_000)
    val, ts, _ = c.rows(g.metric_names)
    g.upload_nodes(val, ts, c.hv, c.hv_ts)
    with pytest.raises(cd.CraneError, match="distinct devices"):
        g.schedule(int(c.now[0]), int(c.now[0]), c.now, c.ds)  # "collective" 1 with n > 1: RCCL
    g.set_option("collective", 0)
    assert g.shard(3)[1:] == (3, 3)
    now = int(c.now[0])
    ch, _ = g.schedule(now, now, c.now, c.ds)
    # (a batch takes its hot values from the binding log at `now`: none uploaded, all 0)
    _, _, och = oracle_soa(spec, c, want_matrix=False,
                           hv_override=(np.zeros(c.n_nodes), np.full(c.n_nodes, now, np.int64)))
    assert np.array_equal(ch, och)
    g.close()


def test_group_through_cpp_driver(tmp_path):
    """The C ABI group from C++ (tests/cpp/plugin_driver.cpp): the snapshot's annotation strings
    parsed by the driver, a one-device group with the one-rank RCCL all-reduce, bindings by global
    index, one batch -> the oracle's chosen nodes; and three shards on the one device."""
    from test_plugin_cpp import LIB_DIR, write_policy
    exe = str(tmp_path / "plugin_driver")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "plugin_driver.cpp"), "-L", LIB_DIR, "-lcrane_dyn",
                    "-Wl,-rpath," + LIB_DIR, "-o", exe], check=True)
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 700, 96, n_bindings=5000, seed=31, pod_step_ns=2_000_000_000, ds_frac=0.1)
    ann = c.annotations()
    now = int(c.now[0])
    base = [f"policy\t{write_policy(tmp_path, spec)}"]
    for i, a in enumerate(ann):
        base.append(f"node\tnode-{i}")
        base += [f"anno\t{k}\t{v}" for k, v in a.items()]
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, now // 10**9)
    _, _, och = oracle_soa(spec, c, want_matrix=False,
                           hv_override=(hv.astype(np.float64), np.full(c.n_nodes, now, np.int64)))
    for devs, coll, threads in (("0", 2, 1), ("0", 2, 0), ("0,0,0", 0, 1)):
        lines = base + [f"group\t{devs}\t2\t{coll}\t{threads}"]
        lines += [f"gbind\t{int(n)}\t{int(t)}" for n, t in zip(c.b_node, c.b_ts)] + ["gbinds"]
        lines += [f"gpod\t{int(t)}\t{int(d)}" for t, d in zip(c.now, c.ds)] + [f"gsched\t{now}"]
        lines += [f"gshard\t{i}" for i in range(devs.count(",") + 1)]
        env = dict(os.environ, TZ="Asia/Shanghai")
        r = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=300,
                           check=True, env=env)
        out = [ln.split("\t") for ln in r.stdout.splitlines()]
        assert not [o for o in out if o[0] == "GERR"], out
        got = np.array([int(o[2]) for o in out if o[0] == "G"])
        assert np.array_equal(got, och), (devs, coll, threads)
        gs = [o for o in out if o[0] == "GS"]
        n = len(gs)
        assert [(int(o[3]), int(o[4])) for o in gs] == [shard.shard_range(c.n_nodes, n, i) for i in range(n)]


def test_forget_stream_before_destroying_it():
    """A caller stream handed back with crane_dyn_forget_stream may be destroyed before the engine's
    next state change (which then does not wait on the dangling handle); destroy syncs the device."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 5000, 500, seed=9, pod_step_ns=1_000_000)
    eng = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    hip = ctypes.CDLL("libamdhip64.so.7")
    dev = torch.device("cuda", 0)
    d_now, d_flags = torch.from_numpy(c.now).to(dev), torch.from_numpy(c.ds).to(dev)
    keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    _, _, och = oracle_soa(spec, c, want_matrix=False)
    for forget in (True, False):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        eng.eval_keys_async(d_now, d_flags, keys, s.value)
        if forget:
            eng.forget_stream(s.value)
            assert np.array_equal(np.array([cd.key_node(int(k))[0] for k in keys.cpu().numpy()]), och)
            assert hip.hipStreamDestroy(s) == 0
            eng.upload_nodes(val, ts, c.hv, c.hv_ts)  # a state change: no wait on the destroyed stream
        else:
            torch.cuda.synchronize()
            assert hip.hipStreamDestroy(s) == 0
    eng.close()  # (the second stream was destroyed without forget: destroy waits for the device only)


@pytest.mark.slow
def test_group_queues_config3_advancing_batch_times():
    """The bench's headline path at full size: BASELINE config 3 (100k nodes x 10k pods, a
    1M-entry binding log) through the group on dispatch queues (depth 4, one device, no
    collective), six batches whose `now` advances by the pods' span (the hot-value cutoffs move
    every batch, each slot sees a different time than its previous batch), all in flight before
    one sync.  Every batch: all keys == one engine stepped on a HIP stream, and a 32-pod sample's
    chosen node and score == the oracle with the binding log's hot values at that batch's now.
    Reference: plugins.go:39-98 + selectHost; binding.go:81-97."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 100_000, 10_000, n_bindings=1_000_000, seed=20250215 + 3000)
    c.now, c.ds = synth.make_pods(10_000, seed=20250215 + 3)
    dev = torch.device("cuda", 0)
    g = cd.Group(cd.Policy(spec), devices=[0], depth=4)
    g.set_option("collective", 0)
    g.set_option("dispatch", 1)
    val, ts, ok = c.rows(g.metric_names)
    g.upload_nodes(val, ts, c.hv, c.hv_ts)
    g.upload_bindings(c.b_node, c.b_ts)
    span = int(c.now[-1] - c.now[0]) + int(c.now[1] - c.now[0])
    times = [int(c.now[0]) + j * span for j in (0, 1, 2, 3, 4, 5)]
    pods = [c.now + j * span for j in range(6)]
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_now = [torch.from_numpy(p).to(dev) for p in pods]
    keys = [torch.empty(len(c.now), dtype=torch.int64, device=dev) for _ in range(6)]
    for b in range(6):  # batch b on slot b % 4; six key buffers, so every batch's keys survive
        g.step_keys_async(times[b], times[b], [d_now[b]], [d_flags], [keys[b]])
    g.sync()
    eng = cd.Engine(cd.Policy(spec), 0)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    eng.upload_bindings(c.b_node, c.b_ts)
    st = torch.cuda.Stream(dev)
    ref = torch.empty_like(keys[0])
    smp = np.unique(np.concatenate([np.linspace(0, 9999, 24).astype(int), np.flatnonzero(c.ds)[:8]]))
    for b in range(6):
        eng.step_keys_async(times[b], times[b], d_now[b], d_flags, ref, st.cuda_stream)
        st.synchronize()
        got = keys[b].cpu().numpy()
        assert np.array_equal(got, ref.cpu().numpy()), f"batch {b}: queue group keys differ from the stream engine's"
        _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, times[b] // 10**9)
        off, osc, och = oracle_soa(spec, c, now=pods[b][smp], ds=c.ds[smp],
                                   hv_override=(hv.astype(np.float64), np.full(c.n_nodes, times[b], np.int64)))
        node, score = shard.unpack_keys(got[smp])
        assert np.array_equal(node, och), f"batch {b}"
        for i in range(len(smp)):
            feas = (off[i] < 0) | (c.ds[smp[i]] != 0)
            assert score[i] == (osc[i][feas].max() if feas.any() else -1), (b, i)
    eng.close()
    g.close()
