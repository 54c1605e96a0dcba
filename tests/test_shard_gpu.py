"""Node sharding through real engines: S engines on one GPU, each holding a
contiguous node range (node_offset) and only its own nodes' bindings, combined
by a host max over their packed keys (the RCCL MAX all-reduce's operation),
equal the unsharded engine and the oracle — with forced equal-score ties across
shard boundaries, whose winner must be the lowest GLOBAL index (key packing
(score << 32) | (0xFFFFFFFF - global node), step.hip / matrix.hip).
Reference: plugins.go:39-98 + upstream selectHost; binding.go:81-97."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

cd = pytest.importorskip("crane_dyn")
from crane_dyn import shard, synth  # noqa: E402
from helpers import oracle_soa  # noqa: E402


def _tied_cluster(n_nodes, n_pods, seed, n_bind):
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, n_nodes, n_pods, n_bindings=n_bind, seed=seed, pod_step_ns=3_000_000)
    # copies of node 3 in later shards: equal metrics, equal hot values
    for dst in (n_nodes // 2 + 1, n_nodes - 5):
        c.val[:, dst], c.ts[:, dst], c.ok[:, dst] = c.val[:, 3], c.ts[:, 3], c.ok[:, 3]
        c.hv[dst], c.hv_ts[dst] = c.hv[3], c.hv_ts[3]
    # every metric fresh and low on the copies: they are among the best nodes
    for n in (3, n_nodes // 2 + 1, n_nodes - 5):
        c.val[:, n], c.ok[:, n], c.ts[:, n] = 0.0, 1, synth.NOW0_NS
        c.hv[n], c.hv_ts[n] = 0.0, synth.NOW0_NS
    return spec, c


@pytest.mark.parametrize("S,keys_path", [(8, 0), (3, 0), (8, 1)])
def test_sharded_engines_equal_unsharded(S, keys_path):
    import torch
    n_nodes, n_pods = 40_003, 2_500
    spec, c = _tied_cluster(n_nodes, n_pods, 20260 + S, 0)
    dev = torch.device("cuda", 0)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    pol = cd.Policy(spec)
    full = cd.Engine(pol, 0)
    val, ts, _ = c.rows(full.metric_names)
    full.upload_nodes(val, ts, c.hv, c.hv_ts)
    ref = torch.empty(n_pods, dtype=torch.int64, device=dev)
    full.eval_keys_async(d_now, d_flags, ref)
    combined = torch.full((n_pods,), -1, dtype=torch.int64, device=dev)
    for r in range(S):
        se = shard.ShardedEngine(pol, n_nodes, S, r, 0)
        se.engine.set_option("keys_path", keys_path)
        se.upload(val, ts, c.hv, c.hv_ts)
        k = torch.empty(n_pods, dtype=torch.int64, device=dev)
        se.eval_keys(d_now, d_flags, k)
        torch.cuda.synchronize()
        combined = torch.maximum(combined, k)
        se.close()
    torch.cuda.synchronize()
    assert torch.equal(combined, ref)
    node, score = shard.unpack_keys(combined.cpu().numpy())
    _, _, och = oracle_soa(spec, c, want_matrix=False)
    assert np.array_equal(node, och)
    assert (node == 3).sum() > 0  # the tie across shards was decided for the lowest global index
    assert not np.isin(node, [n_nodes // 2 + 1, n_nodes - 5]).any()


def test_sharded_step_with_binding_logs():
    """Each shard counts only its own nodes' bindings (re-indexed locally, ShardedEngine.upload):
    the combined step_keys equals the unsharded step and the oracle with binding-log hot values."""
    import torch
    from oracle import oracle as O
    n_nodes, n_pods, S = 30_011, 3_000, 8
    spec, c = _tied_cluster(n_nodes, n_pods, 777, 300_000)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    pol = cd.Policy(spec)
    now = int(synth.NOW0_NS)
    full = cd.Engine(pol, 0)
    val, ts, _ = c.rows(full.metric_names)
    full.upload_nodes(val, ts, c.hv, c.hv_ts)
    full.upload_bindings(c.b_node, c.b_ts)
    ref = torch.empty(n_pods, dtype=torch.int64, device=dev)
    full.step_keys_async(now, now, d_now, d_flags, ref, st.cuda_stream)
    combined = torch.full((n_pods,), -1, dtype=torch.int64, device=dev)
    shards = [shard.ShardedEngine(pol, n_nodes, S, r, 0) for r in range(S)]
    for se in shards:
        se.upload(val, ts, c.hv, c.hv_ts, c.b_node, c.b_ts)
    for rep in range(2):
        ks = []
        for se in shards:
            k = torch.empty(n_pods, dtype=torch.int64, device=dev)
            se.step_keys(now, now, d_now, d_flags, k, st.cuda_stream)
            ks.append(k)
        st.synchronize()
        combined = torch.stack(ks).max(0).values
        assert torch.equal(combined, ref), rep
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, n_nodes, now // 10**9)
    _, _, och = oracle_soa(spec, c, want_matrix=False, hv_override=(hv.astype(np.float64),
                                                                   np.full(n_nodes, now, np.int64)))
    node, _ = shard.unpack_keys(combined.cpu().numpy())
    assert np.array_equal(node, och)
    for se in shards:
        se.close()


_TWO_PROC = dict(n_nodes=30_011, n_pods=3_000, seed=901, n_bind=300_000)


def _two_proc_worker(rank, world, port, out, own_stream=True, backend="gloo"):
    """One rank: a ShardedEngine on GPU 0 holding its node range and those nodes' bindings,
    then ShardedEngine.schedule (local step + MAX all-reduce over gloo, or RCCL at world 1) on
    a stream of the caller's or (own_stream False) with stream=None."""
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    spec, c = _tied_cluster(_TWO_PROC["n_nodes"], _TWO_PROC["n_pods"], _TWO_PROC["seed"], _TWO_PROC["n_bind"])
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    se = shard.ShardedEngine(cd.Policy(spec), c.n_nodes, world, rank, 0)
    val, ts, _ = c.rows(se.engine.metric_names)
    se.upload(val, ts, c.hv, c.hv_ts, c.b_node, c.b_ts)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    now = int(synth.NOW0_NS)
    for rep in range(2):  # the second step re-runs K2 on the same log (idempotent)
        if own_stream:
            se.schedule(now, now, d_now, d_flags, d_keys, st.cuda_stream)
        else:  # torch's current stream: the keys are read there right after
            d_keys.fill_(-7)
            se.schedule(now, now, d_now, d_flags, d_keys)
        if rank == 0:
            np.save(f"{out}.{rep}.npy", d_keys.cpu().numpy())
    dist.barrier()
    se.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,own_stream,backend", [(2, True, "gloo"), (2, False, "gloo"), (1, False, "nccl")])
def test_two_process_sharded_schedule(tmp_path, world, own_stream, backend):
    """Two processes on GPU 0 (one per rank, as bench.py --gpus 2 runs them), each with a
    ShardedEngine over half the nodes, combined by ShardedEngine.schedule's all-reduce: the
    keys equal one engine over the whole cluster, and its chosen nodes equal the oracle's.
    stream=None orders the step and the collective after torch's current stream and before
    its next read; RCCL runs at world size 1 (one GPU: two RCCL ranks cannot share it)."""
    import socket

    import torch
    import torch.multiprocessing as mp
    from oracle import oracle as O

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "keys")
    mp.start_processes(_two_proc_worker, args=(world, port, out, own_stream, backend), nprocs=world,
                       start_method="spawn")
    spec, c = _tied_cluster(_TWO_PROC["n_nodes"], _TWO_PROC["n_pods"], _TWO_PROC["seed"], _TWO_PROC["n_bind"])
    dev = torch.device("cuda", 0)
    full = cd.Engine(cd.Policy(spec), 0)
    val, ts, _ = c.rows(full.metric_names)
    full.upload_nodes(val, ts, c.hv, c.hv_ts)
    full.upload_bindings(c.b_node, c.b_ts)
    now = int(synth.NOW0_NS)
    ref = torch.empty(len(c.now), dtype=torch.int64, device=dev)
    full.step_keys_async(now, now, torch.from_numpy(c.now).to(dev), torch.from_numpy(c.ds).to(dev), ref)
    torch.cuda.synchronize()
    ref = ref.cpu().numpy()
    full.close()
    for rep in range(2):
        assert np.array_equal(np.load(f"{out}.{rep}.npy"), ref), rep
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, c.n_nodes, now // 10**9)
    _, _, och = oracle_soa(spec, c, want_matrix=False, hv_override=(hv.astype(np.float64),
                                                                   np.full(c.n_nodes, now, np.int64)))
    node, _ = shard.unpack_keys(ref)
    assert np.array_equal(node, och)
    assert (node == 3).sum() > 0


def test_config4_global_combine_full_size():
    """BASELINE config 4 at full size on one GPU: 1M nodes x 100k pods split into 8 node shards
    (125k nodes each, node_offset, each with its own nodes' bindings from the one 1M-entry
    log), every shard's step keys max-combined (the RCCL MAX all-reduce's operation) equal
    one engine holding the whole 1M-node cluster, and a 64-pod sample equals the oracle with
    the binding-log hot values.  Reference: plugins.go:39-98 + selectHost, binding.go:81-97;
    SURVEY 8(e)."""
    import torch
    from oracle import oracle as O
    cfg = synth.CONFIGS[4]
    spec = cd.default_policy_spec()
    N, P, S = cfg["nodes"], cfg["pods"], 8
    c = synth.make_cluster(spec, N, P, n_bindings=cfg["bindings"], seed=20250215 + 4000)
    c.now, c.ds = synth.make_pods(P, seed=20250215 + 4)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    pol = cd.Policy(spec)
    now = int(synth.NOW0_NS)
    full = cd.Engine(pol, 0)
    val, ts, _ = c.rows(full.metric_names)
    full.upload_nodes(val, ts, c.hv, c.hv_ts)
    full.upload_bindings(c.b_node, c.b_ts)
    ref = torch.empty(P, dtype=torch.int64, device=dev)
    full.step_keys_async(now, now, d_now, d_flags, ref, st.cuda_stream)
    st.synchronize()
    full.close()
    combined = torch.full((P,), -1, dtype=torch.int64, device=dev)
    k = torch.empty(P, dtype=torch.int64, device=dev)
    for r in range(S):
        se = shard.ShardedEngine(pol, N, S, r, 0)
        se.upload(val, ts, c.hv, c.hv_ts, c.b_node, c.b_ts)
        se.step_keys(now, now, d_now, d_flags, k, st.cuda_stream)
        st.synchronize()
        combined = torch.maximum(combined, k)
        se.close()
    assert torch.equal(combined, ref)
    node, score = shard.unpack_keys(combined.cpu().numpy())
    sample = np.unique(np.concatenate([np.arange(8), np.linspace(0, P - 1, 48).astype(int),
                                       np.flatnonzero(c.ds)[:8]]))[:64]
    _, hv = O.hot_values(spec, c.b_node, c.b_ts, N, now // 10**9)
    _, _, och = oracle_soa(spec, c, now=c.now[sample], ds=c.ds[sample], want_matrix=False, threads=16,
                           hv_override=(hv.astype(np.float64), np.full(N, now, np.int64)))
    assert np.array_equal(node[sample], och)
