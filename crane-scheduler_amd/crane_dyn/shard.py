"""Node sharding across GPUs: one engine per rank, one int64 MAX all-reduce per pod batch.

Each rank owns a contiguous node range [lo, hi) (uploaded with node_offset=lo,
so keys carry GLOBAL node indices).  A per-pod key packs (score, node):
    key = (score << 32) | (0xFFFFFFFF - global_node),   -1 = no feasible node
so max(key) is the highest score with the lowest global node index — the
same tie-break on every shard layout.  torch.distributed with the "nccl"
backend is RCCL on ROCm (xGMI); "gloo" runs the same protocol on CPU.
"""
from __future__ import annotations

import numpy as np

NO_NODE = -1


def shard_range(n_nodes: int, world: int, rank: int):
    """Contiguous, balanced node range of `rank` (first n % world ranks get one extra)."""
    q, r = divmod(n_nodes, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def pack_keys(chosen_global, chosen_score):
    """Host-side packing identical to the device's (engine crane_dyn_eval_keys_async)."""
    ch = np.asarray(chosen_global, np.int64)
    sc = np.asarray(chosen_score, np.int64)
    keys = (sc << 32) | (np.int64(0xFFFFFFFF) - ch)
    return np.where(ch < 0, np.int64(NO_NODE), keys)


def unpack_keys(keys):
    k = np.asarray(keys, np.int64)
    node = np.where(k < 0, -1, np.int64(0xFFFFFFFF) - (k & 0xFFFFFFFF))
    score = np.where(k < 0, -1, k >> 32)
    return node, score


def allreduce_keys(keys, group=None):
    """MAX all-reduce of a torch int64 tensor of per-pod keys, in place (RCCL / gloo)."""
    import torch.distributed as dist

    dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=group)
    return keys


class ShardedEngine:
    """One rank's shard: an Engine holding nodes [lo, hi) of a cluster (global indices in
    its keys), the bindings of those nodes, and the combine step."""

    def __init__(self, policy, n_nodes_total, world, rank, device=0):
        from crane_dyn import Engine

        self.lo, self.hi = shard_range(n_nodes_total, world, rank)
        self.engine = Engine(policy, device)

    def upload(self, val, ts, hv=None, hv_ts=None, b_node=None, b_ts=None):
        """Full-cluster SoA in; this rank keeps its slice (bindings re-indexed locally)."""
        lo, hi = self.lo, self.hi
        self.engine.upload_nodes(val[:, lo:hi], ts[:, lo:hi], None if hv is None else hv[lo:hi],
                                 None if hv_ts is None else hv_ts[lo:hi], node_offset=lo)
        if b_node is not None:
            m = (b_node >= lo) & (b_node < hi)
            self.engine.upload_bindings((b_node[m] - lo).astype(np.int32), b_ts[m])

    def step_keys(self, now_ns, hv_ts_ns, d_now, d_flags, d_keys, stream=None):
        """This shard's keys for the pod batch: hot values from its bindings, then Filter + Score + argmax."""
        self.engine.step_keys_async(now_ns, hv_ts_ns, d_now, d_flags, d_keys, stream)

    def eval_keys(self, d_now, d_flags, d_keys, stream=None):
        """This shard's keys with the current hot values."""
        self.engine.eval_keys_async(d_now, d_flags, d_keys, stream)

    def schedule(self, now_ns, hv_ts_ns, d_now, d_flags, d_keys, stream=None, group=None):
        """One batch across all ranks: local step, then the MAX all-reduce (the global choice).
        The step and the all-reduce run on one stream: `stream`, or (None) a stream of this
        shard that first waits for torch's current stream (the inputs) and that the current
        stream then waits for (the reduced keys) — the engine's own stream is not ordered with
        torch's, so the collective may not simply follow it.  RCCL ("nccl") reduces the device
        keys in place on that stream; a CPU-only backend (gloo) reduces a host copy, written
        back into d_keys."""
        import torch
        import torch.distributed as dist

        cur = None
        if stream is None:
            cur = torch.cuda.current_stream(d_keys.device)
            if getattr(self, "_stream", None) is None:
                self._stream = torch.cuda.Stream(d_keys.device)
            self._stream.wait_stream(cur)
            stream = self._stream.cuda_stream
        self.step_keys(now_ns, hv_ts_ns, d_now, d_flags, d_keys, stream)
        st = torch.cuda.ExternalStream(stream, device=d_keys.device)
        if dist.get_backend(group) == "nccl":
            with torch.cuda.stream(st):
                allreduce_keys(d_keys, group)
        else:
            st.synchronize()
            h = allreduce_keys(d_keys.cpu(), group)
            with torch.cuda.stream(st):
                d_keys.copy_(h)
        if cur is not None:
            cur.wait_stream(st)
        return d_keys

    def close(self):
        self.engine.close()
