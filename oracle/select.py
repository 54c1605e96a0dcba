"""Framework-level selection restated for the checker.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of crane_dyn_select
(crane-scheduler_amd/csrc/select.hip) — never by the product path.

What kube-scheduler v1.23.3 (k8s.io/kubernetes, reference go.mod:26; not in the
container — restated from its published pkg/scheduler/core/generic_scheduler.go,
so this part is "parity unpinned" by reference tests) does per pod of the queue
around the Dynamic plugin, with the Filter / Score results of every (pod, node)
given as matrices (oracle.eval_soa / eval_strings):

  numFeasibleNodesToFind(N): N if N < minFeasibleNodesToFind (100) or
      percentageOfNodesToScore >= 100; else the adaptive percentage
      50 - N/125 (at least minFeasibleNodesPercentageToFind, 5) when the
      configured one is <= 0; N * pct / 100, at least 100.
  findNodesThatPassFilters: nodes checked in rotated order from
      nextStartNodeIndex until numNodesToFind pass every filter plugin (the
      sequential order of upstream's parallel check), then
      nextStartNodeIndex = (nextStartNodeIndex + processed) % N.
  prioritizeNodes: sum over score plugins of weight * score: Dynamic's
      (plugins.go:73-98) times its weight (scheduler-config.yaml:13-15: 3) plus
      the other plugins' weighted sum per node (ext_score).
  selectHost: the max; ties: lowest node index (tie_seed 0) or the seeded
      bijective tie key of select.hip (upstream: reservoir sampling with
      math/rand — not reproducible, a declared deviation).
DaemonSet pods bypass Dynamic's Filter (plugins.go:41-43) but not the others.
"""
from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF


def num_feasible_nodes_to_find(n: int, percentage: int = 0) -> int:
    if n < 100 or percentage >= 100:
        return n
    pct = percentage
    if pct <= 0:
        pct = max(50 - n // 125, 5)
    k = n * pct // 100
    return max(k, 100)


def _fmix32(x: int) -> int:
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & M32
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & M32
    x ^= x >> 16
    return x


def _splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def tie_keys(seed: int, n_nodes: int, pod: int, node_offset: int = 0) -> np.ndarray:
    """The tie key of every node for one pod (larger wins among equal totals)."""
    g = np.arange(node_offset, node_offset + n_nodes, dtype=np.uint64)
    if seed == 0:
        return (M32 - g).astype(np.uint64)
    kb = ((seed * 0x9E3779B97F4A7C15) & M64) >> 32
    cp = _splitmix64(seed ^ (((pod + 1) * 0xD1B54A32D192ED03) & M64)) & M32
    x = (g ^ np.uint64(kb)) & np.uint64(M32)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & np.uint64(M32)
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & np.uint64(M32)
    x ^= x >> np.uint64(16)
    return x ^ np.uint64(cp)


def framework_select(first_fail, score, ds, ext_ok=None, ext_score=None, dyn_weight=3, percentage=0, start=0,
                     tie_seed=0):
    """first_fail / score: [P][N] Filter (-1 = Success) / Score of the Dynamic plugin.
    Returns chosen[P] (-1: none feasible), total[P] (-1), wstart[P], wlen[P], next_start."""
    first_fail = np.asarray(first_fail)
    score = np.asarray(score, np.int64)
    P, N = first_fail.shape
    ok = np.ones(N, bool) if ext_ok is None else np.asarray(ext_ok).astype(bool)
    ext = np.zeros(N, np.int64) if ext_score is None else np.asarray(ext_score, np.int64)
    K = num_feasible_nodes_to_find(N, percentage)
    chosen = np.full(P, -1, np.int64)
    total = np.full(P, -1, np.int64)
    wstart = np.zeros(P, np.int64)
    wlen = np.zeros(P, np.int64)
    s = int(start)
    for p in range(P):
        feas = ok & ((first_fail[p] < 0) | bool(ds[p]))
        order = (s + np.arange(N)) % N
        if K < N:
            cum = np.cumsum(feas[order])
            hit = np.nonzero(cum == K)[0]
            processed = int(hit[0]) + 1 if len(hit) else N
        else:
            processed = N
        wstart[p], wlen[p] = s, processed
        window = order[:processed]
        cand = window[feas[window]]
        if len(cand):
            tot = dyn_weight * score[p, cand] + ext[cand]
            best = tot.max()
            ties = cand[tot == best]
            tk = tie_keys(int(tie_seed), N, p)[ties]
            chosen[p] = int(ties[int(np.argmax(tk))])
            total[p] = int(best)
        s = (s + processed) % N if N else s
    return chosen, total, wstart, wlen, s
