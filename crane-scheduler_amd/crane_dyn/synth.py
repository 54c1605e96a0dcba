"""Deterministic synthetic clusters for the Dynamic plugin path.

Per node n and metric m (one annotation per syncPolicy metric):
  value  = k/1e5 with k ~ Beta(2,3) * 1.2 rounded to 5 decimals — the domain of
           strconv.FormatFloat(v,'f',5,64) in pkg/controller/prometheus/prometheus.go:124;
  stamp  = now0 - U[0, 1.5 * (period + 5m)) whole seconds, so about a third is stale;
  errors = 2% missing key, 0.5% malformed value, 0.1% negative value.
node_hot_value = int in [0, 12] stamped now0 - U[0, 450) s.
Pods: now_p = now0 + p * 1 ms (time.Now() per call in the reference), 1% DaemonSet.
Binding log (configs 3-5): node ids Zipf(1.1) over N, timestamps monotone in
[now0 - 600, now0] (a ring equals the reference's min-heap only for
time-ordered inserts, binding.go:69-78).
"""
from __future__ import annotations

import dataclasses
import datetime as _dt

import numpy as np

NOW0 = 1792065600  # 2026-10-15T20:00:00+08:00
NOW0_NS = NOW0 * 10**9
TS_INVALID = -(2**63)
SHANGHAI = 8 * 3600

# BASELINE.json configs (index = config id)
CONFIGS = {
    1: dict(nodes=100, pods=1, bindings=0),
    2: dict(nodes=5_000, pods=1_000, bindings=0),
    3: dict(nodes=100_000, pods=10_000, bindings=1_000_000),
    4: dict(nodes=1_000_000, pods=100_000, bindings=1_000_000),
    5: dict(nodes=100_000, pods=50_000, bindings=1_000_000),
}


@dataclasses.dataclass
class Cluster:
    metric_names: list          # syncPolicy metric names (row order of val/ts/ok)
    val: np.ndarray             # [M][N] float64
    ts: np.ndarray              # [M][N] int64 ns, TS_INVALID = missing/malformed
    ok: np.ndarray              # [M][N] uint8, 1 = well-formed annotation
    malformed: np.ndarray       # [M][N] bool
    hv: np.ndarray              # [N] float64 (integer valued)
    hv_ts: np.ndarray           # [N] int64 ns
    now: np.ndarray             # [P] int64 ns
    ds: np.ndarray              # [P] uint8 DaemonSet flag
    b_node: np.ndarray          # [B] int32
    b_ts: np.ndarray            # [B] int64 unix s
    seed: int

    @property
    def n_nodes(self):
        return self.val.shape[1]

    def rows(self, names):
        """val/ts/ok rows in the order of `names` (e.g. an Engine's metric_names)."""
        idx = [self.metric_names.index(n) for n in names]
        return self.val[idx], self.ts[idx], self.ok[idx]

    def node_slice(self, lo, hi):
        c = dataclasses.replace(self)
        c.val, c.ts, c.ok, c.malformed = (x[:, lo:hi] for x in (self.val, self.ts, self.ok, self.malformed))
        c.hv, c.hv_ts = self.hv[lo:hi], self.hv_ts[lo:hi]
        m = (self.b_node >= lo) & (self.b_node < hi)
        c.b_node, c.b_ts = (self.b_node[m] - lo).astype(np.int32), self.b_ts[m]
        c._raw_ts_s = self._raw_ts_s[:, lo:hi]
        return c

    def annotations(self, lo=0, hi=None, tz_offset_s=SHANGHAI):
        """Node annotation dicts exactly as the controller would have written them."""
        hi = self.n_nodes if hi is None else hi
        out = []
        for n in range(lo, hi):
            a = {}
            for m, name in enumerate(self.metric_names):
                if not self.ok[m, n] and not self.malformed[m, n]:
                    continue  # missing key
                stamp = _fmt(self.ts_seconds(m, n), tz_offset_s)
                if self.malformed[m, n]:
                    a[name] = f"{self.val[m, n]:.5f}" if n % 2 else f"n/a,{stamp}"
                else:
                    a[name] = f"{self.val[m, n]:.5f},{stamp}"
            if self.hv_ts[n] != TS_INVALID:
                a["node_hot_value"] = f"{int(self.hv[n])},{_fmt(int(self.hv_ts[n] // 10**9), tz_offset_s)}"
            out.append(a)
        return out

    def ts_seconds(self, m, n):
        t = self.ts[m, n]
        return int(t // 10**9) if t != TS_INVALID else int(self._raw_ts_s[m, n])


def concat(cells):
    """One cluster from node cells laid end to end (cell k's nodes follow cell k-1's; its
    bindings are re-indexed by the cell's offset).  Pods are the first cell's."""
    c = dataclasses.replace(cells[0])
    c.val, c.ts, c.ok, c.malformed = (np.concatenate([getattr(x, f) for x in cells], axis=1)
                                      for f in ("val", "ts", "ok", "malformed"))
    c.hv = np.concatenate([x.hv for x in cells])
    c.hv_ts = np.concatenate([x.hv_ts for x in cells])
    offs = np.cumsum([0] + [x.n_nodes for x in cells[:-1]])
    c.b_node = np.concatenate([x.b_node.astype(np.int64) + o for x, o in zip(cells, offs)]).astype(np.int32)
    c.b_ts = np.concatenate([x.b_ts for x in cells])
    c._raw_ts_s = np.concatenate([x._raw_ts_s for x in cells], axis=1)
    return c


def _fmt(unix_s, off):
    return (_dt.datetime(1970, 1, 1) + _dt.timedelta(seconds=int(unix_s) + off)).strftime("%Y-%m-%dT%H:%M:%SZ")


def make_pods(n_pods, seed, now0=NOW0, ds_frac=0.01, pod_step_ns=1_000_000):
    """A pod batch independent of the node shard: now_p = now0 + p*step, DaemonSet flags."""
    rng = np.random.default_rng(seed)
    now = now0 * 10**9 + np.arange(n_pods, dtype=np.int64) * pod_step_ns
    return now, (rng.random(n_pods) < ds_frac).astype(np.uint8)


def make_cluster(policy_spec, n_nodes, n_pods, n_bindings=0, seed=20250215, now0=NOW0, invalid=True, ds_frac=0.01,
                 pod_step_ns=1_000_000):
    rng = np.random.default_rng(seed)
    names = [n for n, _ in policy_spec["syncPolicy"]]
    periods = np.array([p for _, p in policy_spec["syncPolicy"]], np.int64)
    M, N = len(names), n_nodes
    k = np.round(rng.beta(2.0, 3.0, (M, N)) * 1.2 * 1e5)
    val = k / 1e5
    dur_s = (periods + 300 * 10**9) // 10**9
    age = np.floor(rng.random((M, N)) * (1.5 * dur_s)[:, None]).astype(np.int64)
    ts_s = now0 - age
    ok = np.ones((M, N), np.uint8)
    malformed = np.zeros((M, N), bool)
    if invalid:
        r = rng.random((M, N))
        missing = r < 0.02
        malformed = (r >= 0.02) & (r < 0.025)
        negative = (r >= 0.025) & (r < 0.026)
        val = np.where(negative, -np.maximum(val, 1e-5), val)
        ok[missing | malformed] = 0
    ts = np.where(ok == 1, ts_s * 10**9, TS_INVALID).astype(np.int64)
    val = np.where(ok == 1, val, 0.0)
    hv = rng.integers(0, 13, N).astype(np.float64)
    hv_ts = (now0 - rng.integers(0, 450, N)).astype(np.int64) * 10**9
    now = now0 * 10**9 + np.arange(n_pods, dtype=np.int64) * pod_step_ns
    ds = (rng.random(n_pods) < ds_frac).astype(np.uint8)
    if n_bindings:
        ranks = np.arange(1, N + 1, dtype=np.float64)
        p = ranks ** -1.1
        cdf = np.cumsum(p / p.sum())
        b_rank = np.searchsorted(cdf, rng.random(n_bindings), side="right").clip(0, N - 1)
        perm = rng.permutation(N)
        b_node = perm[b_rank].astype(np.int32)
        b_ts = np.sort(rng.integers(now0 - 600, now0 + 1, n_bindings)).astype(np.int64)
    else:
        b_node = np.zeros(0, np.int32)
        b_ts = np.zeros(0, np.int64)
    c = Cluster(names, val, ts, ok, malformed, hv, hv_ts, now, ds, b_node, b_ts, seed)
    c._raw_ts_s = ts_s
    return c
