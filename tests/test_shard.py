"""Multi-rank protocol on CPU: node shards + int64 MAX all-reduce over gloo (world size 2 and 3).

Per-shard evaluation here is the CPU oracle (the GPU engine computes the same
keys on device); the test checks that sharding, global indices, key packing
and the MAX reduction reproduce the unsharded choice, ties included.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sets sys.path)
from crane_dyn import shard
from crane_dyn import synth


def _spec():
    m = 60 * 10**9
    return {
        "syncPolicy": [("cpu_usage_avg_5m", 3 * m), ("cpu_usage_max_avg_1h", 15 * m), ("cpu_usage_max_avg_1d", 180 * m),
                       ("mem_usage_avg_5m", 3 * m), ("mem_usage_max_avg_1h", 15 * m), ("mem_usage_max_avg_1d", 180 * m)],
        "predicate": [("cpu_usage_avg_5m", 0.65), ("cpu_usage_max_avg_1h", 0.75), ("mem_usage_avg_5m", 0.65),
                      ("mem_usage_max_avg_1h", 0.75)],
        "priority": [("cpu_usage_avg_5m", 0.2), ("cpu_usage_max_avg_1h", 0.3), ("cpu_usage_max_avg_1d", 0.5),
                     ("mem_usage_avg_5m", 0.2), ("mem_usage_max_avg_1h", 0.3), ("mem_usage_max_avg_1d", 0.5)],
        "hotValue": [(5 * m, 5), (1 * m, 2)],
    }


def _local_keys(spec, c, lo, hi):
    from oracle import oracle as O
    s = c.node_slice(lo, hi)
    hv_ok = (s.hv_ts != synth.TS_INVALID).astype(np.uint8)
    ff, sc, _ = O.eval_soa(spec, s.metric_names, s.ok, s.val, np.where(s.ok == 1, s.ts, 0), hv_ok, s.hv, s.hv_ts,
                           c.now, c.ds)
    P = len(c.now)
    ch = np.full(P, -1, np.int64)
    cs = np.full(P, -1, np.int64)
    for p in range(P):
        feas = (ff[p] < 0)
        if feas.any():
            best = np.where(feas, sc[p], -1)
            j = int(np.argmax(best))  # first max = lowest local index
            ch[p], cs[p] = lo + j, best[j]
    return shard.pack_keys(ch, cs)


def _worker(rank, world, port, n_nodes, n_pods, seed, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = _spec()
    c = synth.make_cluster(spec, n_nodes, n_pods, seed=seed, pod_step_ns=2_000_000_000)
    c.val[:, 391] = c.val[:, 3]  # force exact score ties across shards
    c.ts[:, 391] = c.ts[:, 3]
    c.ok[:, 391] = c.ok[:, 3]
    c.hv[391], c.hv_ts[391] = c.hv[3], c.hv_ts[3]
    lo, hi = shard.shard_range(n_nodes, world, rank)
    keys = torch.from_numpy(_local_keys(spec, c, lo, hi))
    shard.allreduce_keys(keys)
    if rank == 0:
        node, score = shard.unpack_keys(keys.numpy())
        np.save(out, np.stack([node, score]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_choice_matches_unsharded(tmp_path, world):
    n_nodes, n_pods, seed = 401, 24, 77
    out = str(tmp_path / "res.npy")
    mp.start_processes(_worker, args=(world, _free_port(), n_nodes, n_pods, seed, out), nprocs=world,
                       start_method="spawn")
    node, score = np.load(out)
    spec = _spec()
    c = synth.make_cluster(spec, n_nodes, n_pods, seed=seed, pod_step_ns=2_000_000_000)
    c.val[:, 391] = c.val[:, 3]
    c.ts[:, 391] = c.ts[:, 3]
    c.ok[:, 391] = c.ok[:, 3]
    c.hv[391], c.hv_ts[391] = c.hv[3], c.hv_ts[3]
    ref_node, ref_score = shard.unpack_keys(_local_keys(spec, c, 0, n_nodes))
    assert node.tolist() == ref_node.tolist()
    assert score.tolist() == ref_score.tolist()


def test_bench_gpus_needs_that_many_gpus():
    """bench.py --gpus N launches N ranks itself, and refuses (instead of timing one rank and
    reporting n_gpus 1) when fewer GPUs are visible — here, none."""
    import subprocess
    import sys
    if torch.cuda.device_count() >= 4:
        pytest.skip("host has >= 4 GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "--gpus 4 needs 4 visible GPUs" in r.stderr


def test_bench_global_cluster_slices():
    """Config-4 shards are slices of ONE global cluster (same arrays at every N), config-3
    cells are the weak-scaling global cluster's node ranges."""
    import argparse
    import bench
    spec = _spec()
    saved = dict(synth.CONFIGS)
    try:
        synth.CONFIGS[4] = dict(nodes=1000, pods=8, bindings=5000)
        synth.CONFIGS[3] = dict(nodes=300, pods=8, bindings=2000)
        for cfg in (3, 4):
            a = argparse.Namespace(config=cfg)
            whole = bench.build_shard(synth, spec, a, 3, 0)[3]()
            for world in (1, 2, 3) if cfg == 4 else (3,):  # (config 3's global cluster grows with N)
                parts = [bench.build_shard(synth, spec, a, world, r) for r in range(world)]
                assert sum(p[0].n_nodes for p in parts) == whole.n_nodes
                for c, lo, n_total, _ in parts:
                    assert n_total == whole.n_nodes
                    hi = lo + c.n_nodes
                    assert np.array_equal(c.val, whole.val[:, lo:hi]) and np.array_equal(c.ts, whole.ts[:, lo:hi])
                    assert np.array_equal(c.hv, whole.hv[lo:hi]) and np.array_equal(c.hv_ts, whole.hv_ts[lo:hi])
                    m = (whole.b_node >= lo) & (whole.b_node < hi)
                    assert np.array_equal(c.b_node, whole.b_node[m] - lo) and np.array_equal(c.b_ts, whole.b_ts[m])
                    assert np.array_equal(c.now, parts[0][0].now)
    finally:
        synth.CONFIGS.clear()
        synth.CONFIGS.update(saved)


def test_shard_ranges_cover():
    for n in (0, 1, 7, 100, 1_000_001):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_key_packing_tiebreak():
    k = shard.pack_keys([5, 3, -1, 4_000_000_000], [90, 90, -1, 100])
    assert k[1] > k[0]  # same score: lower index wins the max
    assert k[2] == -1
    node, score = shard.unpack_keys(k)
    assert node.tolist() == [5, 3, -1, 4_000_000_000] and score.tolist() == [90, 90, -1, 100]


def test_c_shard_range_matches():
    """crane_shard_range (the group's split, group.cpp) equals shard.shard_range."""
    cd = pytest.importorskip("crane_dyn")
    for n in (0, 1, 7, 100, 1_000_001, 2**32 - 1):
        for w in (1, 2, 3, 7, 8):
            for r in range(w):
                assert cd.shard_range(n, w, r) == shard.shard_range(n, w, r)
    with pytest.raises(cd.CraneError):
        cd.shard_range(10, 0, 0)
    with pytest.raises(cd.CraneError):
        cd.shard_range(10, 2, 2)


def test_group_without_gpu_fails_cleanly():
    cd = pytest.importorskip("crane_dyn")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(cd.CraneError):
        cd.Group(cd.Policy(cd.default_policy_spec()), devices=[0])
