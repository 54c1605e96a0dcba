"""Steps on dispatch queues (crane_queue, crane_dyn_step_keys_queue; csrc/aql.cpp): the step's
kernels written as AQL packets by the calling thread instead of HIP launches.  Every test compares
the queue's keys bit for bit with the same engine state stepped on a HIP stream (the path the
oracle tests pin), over advancing batch times so the hot-value cutoffs move, through the kernel
forms that take other launch shapes, fills and fallbacks, past the queue's packet ring, and
through the group (option "dispatch").  The first test checks the oracle directly.
Reference: plugins.go:39-98 + selectHost; binding.go:81-97."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

cd = pytest.importorskip("crane_dyn")
from crane_dyn import synth  # noqa: E402
from helpers import oracle_soa  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _setup(n_nodes, n_pods, n_bind, seed, opts=()):
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, n_nodes, n_pods, n_bindings=n_bind, seed=seed)
    c.now, c.ds = synth.make_pods(n_pods, seed=seed + 1)
    engs = []
    for _ in range(2):
        e = cd.Engine(cd.Policy(spec), 0)
        for k, v in opts:
            e.set_option(k, v)
        val, ts, _ = c.rows(e.metric_names)
        e.upload_nodes(val, ts, c.hv, c.hv_ts)
        e.upload_bindings(c.b_node, c.b_ts)
        engs.append(e)
    dev = torch.device("cuda", 0)
    return spec, c, engs, dev


def _steps_equal(c, engs, dev, times, ring_kind=0):
    """The same batches on engine 0 (HIP stream) and engine 1 (queue): keys equal after each."""
    import torch
    st = torch.cuda.Stream(dev)
    q = cd.Queue(0, ring_kind)
    P = len(c.now)
    for t in times:
        d_now = torch.from_numpy(c.now + (t - synth.NOW0_NS)).to(dev)
        d_flags = torch.from_numpy(c.ds).to(dev)
        torch.cuda.synchronize()
        ka = torch.empty(P, dtype=torch.int64, device=dev)
        kb = torch.empty(P, dtype=torch.int64, device=dev)
        engs[0].step_keys_async(t, t, d_now, d_flags, ka, st.cuda_stream)
        engs[1].step_keys_queue(t, t, d_now, d_flags, kb, q)
        st.synchronize()
        q.wait()
        assert torch.equal(ka, kb), f"queue keys differ from the stream's at t={t}"
    for e in engs:
        e.close()
    q.close()
    return ka.cpu().numpy()


def test_queue_step_equals_stream_and_oracle():
    spec, c, engs, dev = _setup(3000, 700, 20000, 20250301)
    t0 = int(synth.NOW0_NS)
    keys = _steps_equal(c, engs, dev, [t0 + k * 7_000_000_000 for k in (0, 1, 2, 5, 3)] + [t0])
    # the last batch (at t0) against the oracle
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, t0 // 10**9)
    _, _, och = oracle_soa(spec, c, want_matrix=False,
                           hv_override=(hv.astype(np.float64), np.full(c.n_nodes, t0, np.int64)))
    chosen = np.array([cd.key_node(int(k))[0] for k in keys])
    assert np.array_equal(chosen, och)


@pytest.mark.parametrize("opts", [
    (("k2_form", 3),),            # large-form K2 (two kernels, dense buckets; K3p its own launch)
    (("k2_form", 2),),            # atomics K2: a bucket fill between packets (engine stream, waited for)
    (("k1_stream", 0),),          # the record-holding fused node pass
    (("keys_path", 1),),          # per-pair kernel: fills and copies, run on the engine stream
], ids=lambda o: ",".join(f"{k}={v}" for k, v in o))
def test_queue_kernel_forms(opts):
    _, c, engs, dev = _setup(5000, 1500, 40000, 20250302, opts)
    t0 = int(synth.NOW0_NS)
    _steps_equal(c, engs, dev, [t0 + k * 10_000_000_000 for k in (0, 1, 2, 3, 1)])


def test_queue_ring_kinds_and_wrap():
    """Pinned-host kernel arguments, and more packets than the queue's 1024-packet ring."""
    _, c, engs, dev = _setup(2000, 300, 5000, 20250303)
    t0 = int(synth.NOW0_NS)
    _steps_equal(c, engs, dev, [t0 + (k % 7) * 3_000_000_000 for k in range(420)], ring_kind=1)


@pytest.mark.parametrize("threads", [0, 1], ids=["caller-thread", "workers"])
def test_group_dispatch_queues(threads):
    """The group with dispatch 1 (a queue per slot) equals dispatch 0 over slot reuse."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 6000, 1200, n_bindings=30000, seed=20250304)
    c.now, c.ds = synth.make_pods(1200, seed=20250305)
    dev = torch.device("cuda", 0)
    t0 = int(synth.NOW0_NS)
    times = [t0 + (k % 5) * 10_000_000_000 for k in range(23)]
    out = {}
    for dispatch in (0, 1):
        g = cd.Group(cd.Policy(spec), devices=[0], depth=4)
        g.set_option("collective", 0)
        g.set_option("threads", threads)
        g.set_option("dispatch", dispatch)
        val, ts, _ = c.rows(g.metric_names)
        g.upload_nodes(val, ts, c.hv, c.hv_ts)
        g.upload_bindings(c.b_node, c.b_ts)
        d_now = [[torch.from_numpy(c.now + (t - t0)).to(dev)] for t in times]
        d_flags = [torch.from_numpy(c.ds).to(dev)]
        keys = [[torch.empty(len(c.now), dtype=torch.int64, device=dev)] for _ in times]
        torch.cuda.synchronize()
        for b, t in enumerate(times):
            g.step_keys_async(t, t, d_now[b], d_flags, keys[b])
        g.sync()
        out[dispatch] = [k[0].cpu().numpy() for k in keys]
        ch, _ = g.schedule(times[-1], times[-1], c.now + (times[-1] - t0), c.ds)
        out[(dispatch, "schedule")] = ch
        g.close()
    for b in range(len(times)):
        assert np.array_equal(out[0][b], out[1][b]), f"batch {b}"
    assert np.array_equal(out[(0, "schedule")], out[(1, "schedule")])


def test_group_dispatch_refuses_collective():
    """Queues with the PER-BATCH collective are refused (RCCL follows each batch on its HIP stream);
    the batch form takes both (test_group_state_gpu.py)."""
    import torch
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, 500, 64, n_bindings=100, seed=20250306)
    g = cd.Group(cd.Policy(spec), devices=[0], depth=1)
    g.set_option("collective", 2)
    g.set_option("dispatch", 1)
    val, ts, _ = c.rows(g.metric_names)
    g.upload_nodes(val, ts, c.hv, c.hv_ts)
    dev = torch.device("cuda", 0)
    k = torch.empty(64, dtype=torch.int64, device=dev)
    with pytest.raises(cd.CraneError, match="per-batch collective"):
        g.step_keys_async(int(synth.NOW0_NS), int(synth.NOW0_NS), [torch.from_numpy(c.now).to(dev)], None, [k])
    g.close()


def test_forget_queue_then_state_change():
    """A queue handed back (crane_dyn_forget_queue) and destroyed: the engine's next state change
    no longer waits for it; steps on a stream afterwards equal the queue's."""
    import torch
    spec, c, engs, dev = _setup(1500, 200, 3000, 20250307)
    t0 = int(synth.NOW0_NS)
    q = cd.Queue(0)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    torch.cuda.synchronize()
    ka = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    engs[0].step_keys_queue(t0, t0, d_now, d_flags, ka, q)
    assert cd.lib.crane_dyn_forget_queue(engs[0].h, q.h) == 0
    q.close()
    val, ts, _ = c.rows(engs[0].metric_names)
    engs[0].upload_nodes(val, ts, c.hv, c.hv_ts)  # (a state change: waits for its queues — none now)
    st = torch.cuda.Stream(dev)
    kb = torch.empty_like(ka)
    engs[0].step_keys_async(t0, t0, d_now, d_flags, kb, st.cuda_stream)
    st.synchronize()
    assert torch.equal(ka, kb)
    for e in engs:
        e.close()


def test_queue_runs_ahead_past_its_ring():
    """700 steps written to one queue with no wait between them (2,100 packets through a
    1,024-packet ring and its kernarg slots: the writer waits for the packet processor to move on,
    committing its partial step first), then one wait: the last batch's keys equal the stream's."""
    import torch
    _, c, engs, dev = _setup(2000, 300, 5000, 20250308)
    t0 = int(synth.NOW0_NS)
    q = cd.Queue(0)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    torch.cuda.synchronize()
    kq = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    times = [t0 + (k % 5) * 4_000_000_000 for k in range(700)]
    for t in times:
        engs[1].step_keys_queue(t, t, d_now, d_flags, kq, q)
    q.wait()
    st = torch.cuda.Stream(dev)
    ks = torch.empty_like(kq)
    engs[0].step_keys_async(times[-1], times[-1], d_now, d_flags, ks, st.cuda_stream)
    st.synchronize()
    assert torch.equal(kq, ks)
    for e in engs:
        e.close()
    q.close()


@pytest.mark.parametrize("opts", [(), (("k2_form", 3),), (("k2_delta", 0),)], ids=["delta", "large", "dedupe"])
def test_queue_deferred_k3s(opts):
    """Engine option step_defer: a queue step leaves its K3s to the next step on the queue, which
    runs it inside its first launch (with the delta form: k3s_delta_pods; any other first launch
    runs it alone first).  Batches with their own key buffers, one that reuses the previous
    batch's buffer (the deferred K3s runs alone before the new step's K3p resets the keys: the new
    batch's keys must come out whole), a state change in between (the upload runs it first), and
    the last one run by crane_dyn_step_flush: every batch's keys equal the same batch stepped on a
    HIP stream."""
    import torch
    _, c, engs, dev = _setup(5000, 1500, 40000, 20250309, opts)
    engs[1].set_option("step_defer", 1)
    t0 = int(synth.NOW0_NS)
    q = cd.Queue(0)
    st = torch.cuda.Stream(dev)
    P = len(c.now)
    d_flags = torch.from_numpy(c.ds).to(dev)
    times = [t0 + (k % 4) * 9_000_000_000 for k in range(9)]
    d_now = [torch.from_numpy(c.now + (t - t0)).to(dev) for t in times]
    kq = [torch.empty(P, dtype=torch.int64, device=dev) for _ in times]
    kq[5] = kq[4]  # (batch 5 writes batch 4's buffer: batch 4's result is overwritten, batch 5's checked)
    ref = []
    torch.cuda.synchronize()
    for b, t in enumerate(times):
        ks = torch.empty(P, dtype=torch.int64, device=dev)
        engs[0].step_keys_async(t, t, d_now[b], d_flags, ks, st.cuda_stream)
        st.synchronize()
        ref.append(ks)
        if b == 7:  # a state change on the deferring engine between two steps
            val, ts, _ = c.rows(engs[1].metric_names)
            engs[1].upload_nodes(val, ts, c.hv, c.hv_ts)
        engs[1].step_keys_queue(t, t, d_now[b], d_flags, kq[b], q)
    engs[1].step_flush()
    q.wait()
    for b in range(len(times)):
        if b != 4:
            assert torch.equal(kq[b], ref[b]), f"batch {b}"
    for e in engs:
        e.close()
    q.close()
