"""Benchmark of the Dynamic-plugin hot path on MI355X (BASELINE.json configs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3|4] [--no-cpu-baseline] [--no-extras]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Headline (the JSON line's `value`): one step = one scheduling batch of the
reference's hot path over one node shard, keys-only (chosen node per pod):
  K2 hot values from the shard's 1M-entry binding log (binding.go:81-97, node.go:113-121)
  K1 node pass over the shard's parsed annotations (stats.go:51-112 pod-invariant parts)
  K3 Filter + Score + argmax for every (pod, node) pair (plugins.go:39-98, selectHost)
  RCCL int64 max all-reduce of the per-pod packed keys across node shards (N > 1)
Config 3 (default): each GPU owns 100k nodes, all GPUs score the same 10k pods
(weak scaling).  Config 4: the 1M nodes are split over the GPUs, 100k pods
(strong scaling).  `--engine group` (default): one process drives every GPU through
the C ABI group (crane_dyn_group_*: per-device shard engines, in-library RCCL
all-reduce); under a launcher the other ranks only wait.  `--engine ranks`: one
process per GPU over torch.distributed (the comparison).  Batch i is scheduled at
now0 + (i % 6) x 10 s (its pods shifted alike): the hot-value cutoffs move.  `value` is placements per second, measured: the pods of the
timed steps over the timed region.  `pairs_decided_per_s` (P x nodes / step) is
a full-rescan equivalent: every (pod, node) pair's Filter + Score is decided
exactly, but the step path only evaluates a node per pod where one of its
expiries falls inside the batch.  The true per-pair rate (every
pair's result materialised in HBM) is the `matrix_*` legs' `evals_per_s`.
Inputs are resident in HBM before timing; data is synthetic (crane_dyn/synth.py).

Kernel times are the kernels' own dispatch-stamped durations
(crane_dyn_set_profiling), the quantity rocprofv3 --kernel-trace reports.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "crane-scheduler_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
PMC_DIR = os.path.join(ROOT, "profiles", "pmc")
DROPIN = os.path.join(ROOT, "crane-scheduler_amd", "lib", "dropin_bench")
# kernel timer name -> rocprofv3 kernel name (prefix, suffix) for the PMC lookup
# dispatch-stamp name -> (rocprof kernel name without its template arguments, {argument index:
# value}) — the node pass's STEP flag is its 4th template argument, K3m's keys / matrices its
# last two
KERNEL_PMC = {
    "k1_node_pass+k3a_steps": ("crane::k1_node_pass", {3: "true"}),
    "k1_stream_steps": ("crane::k1_stream_steps", {}),
    "k1_node_pass": ("crane::k1_node_pass", {3: "false"}),
    "k2x_dedupe+k3p_pods": ("crane::k2x_dedupe_pods", {}),
    "k2x_dedupe": ("crane::k2x_dedupe", {}),
    "k2_delta+k3p_pods": ("crane::k2_delta_pods", {}),
    "k2_delta": ("crane::k2_delta_pods", {}),
    "k3p_pods": ("crane::k3p_pods", {}),
    "k3s_eval": ("crane::k3s_eval", {}),
    "k3m_matrix+keys": ("crane::k3m_matrix", {-2: "true", -1: "true"}),
    "k3m_matrix": ("crane::k3m_matrix", {-2: "true", -1: "false"}),
}


def pmc_name_match(kname, base, args):
    """rocprof's kernel name kname is `base` (with any template arguments) whose arguments at the
    given positions have the given values."""
    head = kname.split("(", 1)[0]
    tmpl = head[head.index("<") + 1:head.rindex(">")].split(", ") if "<" in head else []
    name = head.split("<", 1)[0]
    return name == base and all(-len(tmpl) <= i < len(tmpl) and tmpl[i] == v for i, v in args.items())


def src_hash():
    """Hash of every source the engine's kernels are built from: PMC summaries are valid for it only."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "crane-scheduler_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "crane-scheduler_amd", "csrc", "*.hpp")) +
                   glob.glob(os.path.join(ROOT, "crane-scheduler_amd", "csrc", "*.cpp")) +
                   glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:12]


def lib_hash():
    """Hash of the engine library file this process loads (an A/B swap shows up here, not in src_hash)."""
    p = os.path.join(ROOT, "crane-scheduler_amd", "lib", "libcrane_dyn.so")
    return hashlib.sha256(open(p, "rb").read()).hexdigest()[:12] if os.path.exists(p) else None


def pmc_summary(config, shash):
    """PMC summary of this config taken on these kernel sources (tools/gpu_pmc.sh), or None."""
    p = os.path.join(PMC_DIR, f"config{config}_{shash}.json")
    return (json.load(open(p)), os.path.relpath(p, ROOT)) if os.path.exists(p) else (None, None)


def k2_path_traffic(ks, by_pos, nread):
    """PMC traffic per launch of one large-form K2 path: k2l_partition of that path (its last
    template argument: ranks by position) + the k2y instantiation the path launched (its first
    argument: regions per lane, the fewest of 2 / 4 / 8 that cover the path's 4096-binding
    regions, hotcount.hip launch_hot_count_large).  ks: a PMC summary's "kernels"."""
    nblk = -(-nread // 4096)
    per = "2" if nblk <= 2048 else "4" if nblk <= 4096 else "8"
    t = [v.get("traffic_bytes") for k, v in ks.items()
         if pmc_name_match(k, "crane::k2l_partition", {-1: "true" if by_pos else "false"})
         or pmc_name_match(k, "crane::k2y_bin_hist", {0: per})]
    return int(sum(t)) if len(t) == 2 and all(x is not None for x in t) else None


def pmc_traffic(pmc, name):
    if not pmc or name not in KERNEL_PMC:
        return None
    base, args = KERNEL_PMC[name]
    hits = [v for k, v in pmc.get("kernels", {}).items() if pmc_name_match(k, base, args) and "traffic_bytes" in v]
    return int(hits[0]["traffic_bytes"]) if hits else None


def effective_cpus():
    """CPUs this process may use: its affinity mask, capped by a cgroup v2 quota."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def task_cpu():
    """{tid: (thread name, CPU seconds)} of this process's threads (/proc/self/task)."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            st = open(f"/proc/self/task/{tid}/stat").read()
            name = st[st.index("(") + 1:st.rindex(")")]
            f = st[st.rindex(")") + 2:].split()
            out[int(tid)] = (name, (int(f[11]) + int(f[12])) / tick)  # utime + stime
        except (OSError, ValueError, IndexError):
            pass
    return out


def host_threads(c0, c1, t_enq, tc_enq, elapsed, steps):
    """Host side of the timed loop: the enqueuing thread's wall and CPU time per step, and the
    other threads of the process that used CPU meanwhile (e.g. a communicator's progress thread
    beside the enqueuing thread; 10 ms tick resolution)."""
    main = threading.get_native_id()
    others = sorted(((c1[t][1] - c0.get(t, (None, 0.0))[1], c1[t][0]) for t in c1 if t != main), reverse=True)
    return {"enqueue_us_per_step": round(t_enq * 1e6 / steps, 2),
            "enqueue_cpu_us_per_step": round(tc_enq * 1e6 / steps, 2),
            "other_threads_cpu_ms": [[n, round(s * 1e3, 1)] for s, n in others[:6] if s > 0],
            "elapsed_ms": round(elapsed * 1e3, 3)}


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def roof(alg_bytes, ms, what, traffic=None, extra=None):
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(gbs / HBM_PEAK_GBS, 4), "ms": round(ms, 4), "alg_bytes": int(alg_bytes), "bytes": what,
         "traffic": traffic}
    if extra:
        r.update(extra)
    return r


def rec_bytes(spec):
    """sizeof(NodeRec<PD, PR>) of the policy's record shape (dyn_types.hpp)."""
    pd_, pr_ = len(spec["predicate"]), len(spec["priority"])
    pd_, pr_ = (4, 6) if pd_ <= 4 and pr_ <= 6 else ((8, 8) if pd_ <= 8 and pr_ <= 8 else (16, 16))
    return -(-(24 + 16 * pr_ + 8 * pd_) // 16) * 16


def delta_changed(spec, b_ts, nows):
    """The delta form's work per batch (engine option k2_delta): bindings whose window rank at the
    batch's time differs from the anchor refresh's (the first batch time: a slot's anchor), i.e. the
    merged ranges between the windows' suffix starts, for each of the timed batches' times."""
    trs = sorted(tr // 10**9 for tr, _ in spec["hotValue"])

    def starts(now_ns):
        cut = np.sort(np.array([now_ns // 10**9 - t for t in trs], np.int64))
        return np.searchsorted(b_ts, cut, side="right")

    a = starts(nows[0])
    ls = []
    for n in nows:
        p = starts(n)
        rg = sorted((min(x, y), max(x, y)) for x, y in zip(a, p) if x != y)
        tot, end = 0, -1
        for lo, hi in rg:
            lo = max(lo, end)
            if hi > lo:
                tot += hi - lo
            end = max(end, hi)
        ls.append(tot)
    return {"per_time": [int(x) for x in ls], "mean": float(np.mean(ls)), "anchor_now_ns": int(nows[0])}


def kernel_times(eng, fn, reps):
    """Mean dispatch-stamped duration per kernel name over `reps` calls of fn()."""
    acc = {}
    eng.set_profiling(True)
    for _ in range(reps):
        fn()
        for name, t in eng.stage_times():
            acc.setdefault(name, []).append(t)
    eng.set_profiling(False)
    return {k: float(np.mean(v)) for k, v in acc.items()}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=8,
                    help="untimed batches first: two per batch slot, so every slot has anchored its hot-value "
                         "counts (delta form) and sized its scratch before the timed region")
    ap.add_argument("--config", type=int, default=3, choices=(3, 4))
    ap.add_argument("--cpu-pods", type=int, default=1920, help="pods in the bounded CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16, help="upstream kube-scheduler parallelism")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-greedy", action="store_true", help="skip the config-5 sequential-greedy measurement")
    ap.add_argument("--inflight", type=int, default=4,
                    help="independent pod batches in flight (engines x HIP streams); 1 = one batch at a time")
    ap.add_argument("--ar-group", type=int, default=0,
                    help="with the collective: batches per keys all-reduce (ranks: a multiple of --inflight, 0 = "
                         "16 x inflight; group: 0 = min(steps, 64))")
    ap.add_argument("--rehearse-collective", action="store_true",
                    help="run the ranks path's N>1 collective on one rank (under torchrun)")
    ap.add_argument("--no-extras", action="store_true", help="headline step only (matrix / drop-in / controller legs off)")
    ap.add_argument("--leg", default="all", choices=("all", "matrix2", "matrix3", "cold"),
                    help="matrix2 / matrix3 / cold: only that leg (for per-kernel PMC passes)")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold-cache 4M-node K1/K2 roofline leg")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option name=value (A/B of kernel forms; repeatable): the --leg runs and the group step")
    ap.add_argument("--group-collective", type=int, default=1, choices=(0, 1, 2),
                    help="group engine: 1 RCCL max all-reduce when n > 1, 2 always (rehearses it on one device), 0 never")
    ap.add_argument("--group-threads", type=int, default=-1, choices=(-1, 0, 1),
                    help="group engine: -1 auto (a worker per device when n > 1), 0 the caller's thread, 1 workers")
    ap.add_argument("--group-dispatch", type=int, default=-1, choices=(-1, 0, 1),
                    help="group engine: 1 the steps' kernels as AQL packets on dispatch queues (crane_queue), "
                         "0 HIP launches on the slots' streams, -1 auto (queues; with the collective the batch form "
                         "orders one all-reduce per window of batches after them)")
    ap.add_argument("--engine", default="group", choices=("group", "ranks"),
                    help="group: one process drives every GPU through the C ABI group (crane_dyn_group_*, "
                         "in-library RCCL); ranks: one process per GPU under torch.distributed (comparison)")
    ap.add_argument("--now-cycle", type=int, default=6,
                    help="timed batch i is scheduled at now0 + (i %% C) x the batch's span (1 = every batch at now0)")
    return ap.parse_args()


# ------------------------------------------------------------------ legs
def select_leg(cd, spec, dev, stream, val, ts, hv, hv_ts, now, ds, reps=3, opts=()):
    """Framework-level selection for the config-3 queue with the shipped profile (SURVEY §8f
    row 4): Dynamic weight 3 + synthetic other plugins (95 % pass their filters, weighted
    sum in [0, 700]), percentageOfNodesToScore default (adaptive: 5 % of 100k = 5000
    feasible nodes per pod from a rotating start) and every node scored (100)."""
    N, P = val.shape[1], len(now)
    eng = cd.Engine(cd.Policy(spec), dev.index)
    for o in opts:
        k, v = o.split("=")
        eng.set_option(k, int(v))
    eng.upload_nodes(val, ts, hv, hv_ts)
    rng = np.random.default_rng(77)
    d_now = torch.from_numpy(now).to(dev)
    d_flags = torch.from_numpy(ds).to(dev)
    d_ok = torch.from_numpy((rng.random(N) < 0.95).astype(np.uint8)).to(dev)
    d_ext = torch.from_numpy(rng.integers(0, 8, N).astype(np.int64) * 100).to(dev)
    ch = torch.empty(P, dtype=torch.int64, device=dev)
    tot = torch.empty(P, dtype=torch.int64, device=dev)
    sh = stream.cuda_stream
    out = {"workload": f"config3 queue: {P} pods x {N} nodes, shipped profile (Dynamic weight 3 + other plugins' "
                       "filter / weighted score per node), lowest-index ties", "parity": "tests/test_select.py"}
    for label, pct in (("adaptive_percentage", 0), ("percentage_100", 100)):
        def step():
            return eng.select(d_now, d_flags, ch, tot, d_ok, d_ext, 3, pct, 0, 0, stream=sh)
        step()
        t0 = time.perf_counter()
        for _ in range(reps):
            nxt = step()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        kt = kernel_times(eng, step, 2)
        out[label] = {"nodes_per_pod": int(cd.num_feasible_nodes_to_find(N, pct)), "ms": round(ms, 3),
                      "pods_per_s": round(P / (ms * 1e-3), 1), "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
                      "next_start": int(nxt), "placed": int((ch >= 0).sum().item())}
    eng.close()
    return out


def matrix_leg(cd, spec, dev, stream, label, val, ts, hv, hv_ts, now, ds, steps, pmc=None):
    """Per-pair path: the full first-fail and score matrices (int8, [P][N] in HBM) and the
    chosen node of every pod, one K3m launch per batch (node records resident: the node pass
    runs once per snapshot sync)."""
    N, P = val.shape[1], len(now)
    eng = cd.Engine(cd.Policy(spec), dev.index)
    eng.upload_nodes(val, ts, hv, hv_ts)
    d_now = torch.from_numpy(now).to(dev)
    d_flags = torch.from_numpy(ds).to(dev)
    d_ff = torch.empty((P, N), dtype=torch.int8, device=dev)
    d_sc = torch.empty((P, N), dtype=torch.int8, device=dev)
    d_keys = torch.empty(P, dtype=torch.int64, device=dev)
    sh = stream.cuda_stream
    t1 = time.perf_counter()
    eng.node_pass_async(sh)
    stream.synchronize()
    sync_ms = (time.perf_counter() - t1) * 1e3

    def step():
        eng.eval_matrix_async(d_now, d_flags, d_ff, d_sc, d_keys, stream=sh)

    for _ in range(3):
        step()
    stream.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    stream.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    kt = kernel_times(eng, step, max(3, steps // 2))
    # the chosen nodes agree with the keys-only step path on the same batch
    d_k2 = torch.empty(P, dtype=torch.int64, device=dev)
    eng.eval_keys_async(d_now, d_flags, d_k2, sh)
    stream.synchronize()
    same = bool(torch.equal(d_keys, d_k2))
    rec = rec_bytes(spec)
    kname = "k3m_matrix+keys"
    kms = kt.get(kname, ms)
    alg = N * rec + P * (8 + 1 + 8) + 2 * P * N
    r = roof(alg, kms, "node records read once + pod now/flag read + keys + first-fail and score matrices "
                       "(int8) written", pmc_traffic(pmc, kname), {"kernel": kname})
    eff = P * N * 112 / (kms * 1e-3) / 1e9
    out = {"workload": label, "nodes": N, "pods": P, "ms": round(ms, 4), "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
           "evals_per_s": round(P * N / (ms * 1e-3), 1), "kernel_evals_per_s": round(P * N / (kms * 1e-3), 1),
           "placements_per_s": round(P / (ms * 1e-3), 1), "roofline": r,
           "effective_GBps_112B_per_eval": round(eff, 1),
           "node_pass_ms_per_sync": round(sync_ms, 3), "chosen_equal_step_path": same,
           "outputs": "first_fail int8 [P][N], score int8 [P][N], keys int64 [P] (device)"}
    eng.close()
    del d_ff, d_sc
    return out


COLD = dict(nodes=4_000_000, bindings=16_000_000, pods=10_000)


def cold_leg(cd, synth, spec, dev, reps=5, pmc=None, pmc_src=None, opts=()):
    """HBM roofline of the two streaming stages at a size no cache holds (the
    >= 60 % claim is on cold-cache K1 and K2): 4M nodes, a 16M-entry binding log.  Before
    the hot-value refresh (K2) and before the node pass (K1 + the step tables) a 1 GiB
    scratch buffer is READ, which evicts the 256 MiB Infinity Cache and the L2s without
    leaving dirty lines to be written back during the timed kernels.  Times are the kernels'
    dispatch-stamped durations (crane_dyn_set_profiling), median over `reps`.
    Two node passes over the same counts: `k1` the step path's (K1 fused with the step
    tables of the pod batch, the headline step's kernel) and `k1_records` the node pass that
    writes every node's record (what the matrix / greedy / selection / drop-in table paths
    read; one per snapshot sync), each after its own K2 refresh and flush.
    Algorithmic bytes:
      K2 = 12 per binding (node i32 + ts i64 read) + 4 per node and window (counts written)
      K1 = 16 per node and metric (value + ts read) + 4 per node and window (counts read)
           + 8 per node (hot value written)
      K1 records = K1 + the record written (sizeof(NodeRec), 160 B at the default policy)"""
    N, B, P = COLD["nodes"], COLD["bindings"], COLD["pods"]
    c = synth.make_cluster(spec, N, P, n_bindings=B, seed=7)
    c.now, c.ds = synth.make_pods(P, seed=8)
    eng = cd.Engine(cd.Policy(spec), dev.index)
    eng.set_option("k2_delta", 0)  # (every refresh here re-counts: the leg prices the whole suffix pass)
    for o in opts:
        k, v = o.split("=")
        eng.set_option(k, int(v))
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    eng.upload_bindings(c.b_node, c.b_ts)
    del val, ts
    st = torch.cuda.Stream(dev)
    sh = st.cuda_stream
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(P, dtype=torch.int64, device=dev)
    scratch = torch.empty(1 << 27, dtype=torch.int64, device=dev).fill_(1)
    sink = torch.empty(1, dtype=torch.int64, device=dev)
    M, W = len(eng.metric_names), len(spec["hotValue"])
    now = int(synth.NOW0_NS)

    def flush():
        with torch.cuda.stream(st):
            torch.sum(scratch, dim=0, keepdim=True, out=sink)

    k2, k1, k1r, k2_parts, k1_parts = [], [], [], {}, {}
    for r in range(reps + 1):
        flush()
        eng.set_profiling(True)
        eng.refresh_hot_values_async(now, now, sh)
        t_k2 = eng.stage_times()
        flush()
        eng.set_profiling(True)
        eng.eval_keys_async(d_now, d_flags, d_keys, sh)
        t_ev = eng.stage_times()
        eng.refresh_hot_values_async(now, now, sh)  # (counts pending again for the record pass)
        flush()
        eng.set_profiling(True)
        eng.node_pass_async(sh)
        t_np = eng.stage_times()
        if r:  # rep 0 warms the code paths
            k2.append(sum(t for _, t in t_k2))
            for name, t in t_k2:
                k2_parts.setdefault(name, []).append(t)
            # the node pass that builds the step tables (one fused kernel: the streamed step pass
            # past the dedupe form's cap, or the record-holding one)
            k1.append(sum(t for name, t in t_ev if name.startswith(("k1_node_pass", "k1_stream_steps"))))
            for name, t in t_ev:
                if name.startswith(("k1_node_pass", "k1_stream_steps")):
                    k1_parts.setdefault(name, []).append(t)
            k1r.append(sum(t for name, t in t_np if name == "k1_node_pass"))
    # the general form for a log in no particular order: every binding's node id and stamp read
    eng.set_option("k2_sorted", 0)
    k2ts, k2ts_parts = [], {}
    for r in range(reps + 1):
        flush()
        eng.set_profiling(True)
        eng.refresh_hot_values_async(now, now, sh)
        t_k2 = eng.stage_times()
        eng.node_pass_async(sh)  # (consume the counts)
        if r:
            k2ts.append(sum(t for _, t in t_k2))
            for name, t in t_k2:
                k2ts_parts.setdefault(name, []).append(t)
    eng.set_profiling(False)
    eng.close()
    del scratch
    k2_ms, k1_ms, k1r_ms = float(np.median(k2)), float(np.median(k1)), float(np.median(k1r))
    k2ts_ms = float(np.median(k2ts))
    tr_k2 = tr_k2ts = tr_k1 = tr_k1r = None
    if pmc:
        ks = pmc.get("kernels", {})

        kr = k2_read(spec, c.b_ts, now)
        tr_k2, tr_k2ts = k2_path_traffic(ks, True, kr["read"]), k2_path_traffic(ks, False, B)
        tr_k1 = pmc_traffic(pmc, "k1_stream_steps")
        if tr_k1 is None:
            tr_k1 = pmc_traffic(pmc, "k1_node_pass+k3a_steps")
        tr_k1r = pmc_traffic(pmc, "k1_node_pass")
    kb = k2_read(spec, c.b_ts, now)
    alg_k2 = kb["bytes"] + 4 * W * N
    alg_k1 = N * (16 * M + 4 * W + 8)
    rec_b = rec_bytes(spec)
    return {"workload": f"{N} nodes x {B}-entry binding log ({P}-pod batch), default policy",
            "cache": "cold: 1 GiB read between the stages (Infinity Cache + L2 evicted, no dirty lines)",
            "k2": roof(alg_k2, k2_ms, kb["what"] + " + per-node window counts written (4 B x W)", tr_k2,
                       {"kernels": {k: round(float(np.median(v)), 4) for k, v in k2_parts.items()}}),
            "k2_timestamp_path": roof(12 * B + 4 * W * N, k2ts_ms, "every binding's node id + stamp read (12 B) "
                                      "+ per-node window counts written (4 B x W): the form for a log in no "
                                      "particular order (engine option k2_sorted 0)", tr_k2ts,
                                      {"kernels": {k: round(float(np.median(v)), 4) for k, v in k2ts_parts.items()}}),
            "k1": roof(alg_k1, k1_ms, "SoA (value, ts) read + window counts read + hot value written", tr_k1,
                       {"kernel": "k1_stream_steps (the node pass fused with the step tables, streamed: "
                                  "no record in registers)",
                        "kernels": {k: round(float(np.median(v)), 4) for k, v in k1_parts.items()}}),
            # priced on the same algorithmic bytes as k1; the 160 B record it writes is
            # the engine's own intermediate, reported only as a stream rate beside it
            "k1_records": roof(alg_k1, k1r_ms, "as k1 (the record the pass writes is not algorithmic)", tr_k1r,
                               {"kernel": "k1_node_pass (records: matrix / greedy / selection / drop-in tables)",
                                "stream_GBps_incl_record": round((alg_k1 + N * rec_b) / (k1r_ms * 1e-3) / 1e9, 1),
                                "record_bytes_per_node": rec_b}),
            "traffic_source": pmc_src if (tr_k1 is not None or tr_k2 is not None or tr_k1r is not None) else None}


DROPIN_CPU = os.path.join(ROOT, "oracle", "_build", "dropin_cpu")


def _dropin_files(d, spec, ann, now, ds):
    pol = {"apiVersion": "scheduler.policy.crane.io/v1alpha1", "kind": "DynamicSchedulerPolicy",
           "spec": {"syncPolicy": [{"name": n, "period": f"{p // 10**9}s"} for n, p in spec["syncPolicy"]],
                    "predicate": [{"name": n, "maxLimitPecent": v} for n, v in spec["predicate"]],
                    "priority": [{"name": n, "weight": v} for n, v in spec["priority"]],
                    "hotValue": [{"timeRange": f"{t // 10**9}s", "count": c} for t, c in spec["hotValue"]]}}
    pp = os.path.join(d, "policy.json")
    json.dump(pol, open(pp, "w"))
    sp = os.path.join(d, "snap.tsv")
    with open(sp, "w") as f:
        for i, a in enumerate(ann):
            f.write(f"N\tnode-{i}\n")
            for k, v in a.items():
                f.write(f"A\t{k}\t{v}\n")
    pd = os.path.join(d, "pods.tsv")
    with open(pd, "w") as f:
        for p in range(len(now)):
            f.write(f"P\tpod-{p}\t{int(now[p])}\t{int(ds[p])}\n")
    return pp, sp, pd


def _replay_chosen(cd, spec, c, dev_index, now, ds, log_path, oracle_pods=()):
    """Every pod's chosen node recomputed on the churned cluster: the harness's log (annotation
    patches, nodes joining "J" and leaving "L", by creation index) applied to the snapshot's SoA pod
    by pod, then one engine holding the live nodes in the snapshot's list order (a full upload per
    pod, no incremental path) evaluates the pod; for the pods in `oracle_pods` the CPU oracle too.
    Returns (chosen creation index [P], oracle agreement or None)."""
    from oracle import oracle as O
    eng = cd.Engine(cd.Policy(spec), dev_index)
    names = eng.metric_names
    val, ts, _ = c.rows(names)
    val, ts = val.copy(), ts.copy()
    hv, hv_ts = c.hv.copy(), c.hv_ts.copy()
    row = {n: i for i, n in enumerate(names)}
    events = {}
    with open(log_path) as f:
        for ln in f:
            t = ln.rstrip("\n").split("\t")
            if t[0] in ("J", "L"):
                events.setdefault(int(t[1]), []).append((t[0], int(t[2]), None, None))
            else:
                events.setdefault(int(t[0]), []).append(("P", int(t[1]), t[2], t[3]))
    live = list(range(c.n_nodes))
    chosen, ok_oracle = [], []
    for p in range(len(now)):
        for kind, n, k, v in events.get(p, ()):
            if kind == "J":
                if n >= val.shape[1]:  # room for the joining node: no annotations until its patches
                    extra = n + 1 - val.shape[1]
                    val = np.concatenate([val, np.zeros((len(names), extra))], axis=1)
                    ts = np.concatenate([ts, np.full((len(names), extra), cd.CRANE_TS_INVALID, np.int64)], axis=1)
                    hv = np.concatenate([hv, np.zeros(extra)])
                    hv_ts = np.concatenate([hv_ts, np.full(extra, cd.CRANE_TS_INVALID, np.int64)])
                live.append(n)
            elif kind == "L":
                live.remove(n)
            else:
                x, t = cd.parse_annotation(v, synth_shanghai())
                if k == "node_hot_value":
                    hv[n], hv_ts[n] = x, t
                elif k in row:
                    val[row[k], n], ts[row[k], n] = x, t
        ids = np.array(live, np.int64)
        lv, lt, lh, lht = val[:, ids], ts[:, ids], hv[ids], hv_ts[ids]
        eng.upload_nodes(lv, lt, lh, lht)
        ch = int(eng.eval(now[p:p + 1], ds[p:p + 1])[2][0])
        chosen.append(int(ids[ch]) if ch >= 0 else -1)
        if p in oracle_pods:
            okm = (lt != cd.CRANE_TS_INVALID).astype(np.uint8)
            _, _, och = O.eval_soa(spec, names, okm, lv, np.where(okm == 1, lt, 0),
                                   (lht != cd.CRANE_TS_INVALID).astype(np.uint8), lh, lht, now[p:p + 1],
                                   ds[p:p + 1], threads=16, want_matrix=False)
            ok_oracle.append(int(och[0]) == ch)
    eng.close()
    return np.array(chosen), (all(ok_oracle) if oracle_pods else None)


def synth_shanghai():
    from crane_dyn import synth
    return synth.SHANGHAI


def dropin_runs(spec, ann, now, ds, threads, cpu_pods=0):
    """The drop-in harness runs of dropin_leg (subprocesses only: call it before this process
    touches the GPU, so the harness's queues are the only ones on the device, as in a scheduler
    process — a parent holding a dozen idle queues made the harness's first update after its
    initial sync wait 5-20 ms for the hardware scheduler).  Returns the runs' outputs and the
    temporary directory holding their churn logs (removed by dropin_leg)."""
    d = tempfile.mkdtemp(prefix="crane_dropin_")
    env = dict(os.environ, TZ="Asia/Shanghai")
    pp, sp, pd = _dropin_files(d, spec, ann, now, ds)
    now_long = now[0] + np.arange(len(now), dtype=np.int64) * 10**9
    pd_long = os.path.join(d, "pods_long.tsv")
    with open(pd_long, "w") as f:
        for p in range(len(now)):
            f.write(f"P\tpod-{p}\t{int(now_long[p])}\t{int(ds[p])}\n")
    runs = {"dir": d, "now_long": now_long, "out": {}, "err": None, "cpu": None}
    if not os.path.exists(DROPIN):
        runs["err"] = f"{DROPIN} not built"
        return runs
    for label, scale, ev, pods_f in (("churn_x1", 1.0, 0, pd), ("churn_x10", 10.0, 0, pd), ("frozen", 0.0, 0, pd),
                                     ("nodes_and_time", 1.0, 8, pd_long)):
        lp = os.path.join(d, f"{label}.log")
        cmd = [DROPIN, pp, sp, pods_f, "--threads", str(threads), "--churn", str(scale), "--churn-log", lp,
               "--node-events", str(ev)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
        if os.environ.get("CRANE_DROPIN_STDERR"):  # (diagnostics: the harness's stderr per run)
            with open(f"{os.environ['CRANE_DROPIN_STDERR']}_{label}.txt", "w") as f:
                f.write(r.stderr)
        if r.returncode != 0:
            runs["err"] = f"{label}: {r.stderr[-500:]}"
            return runs
        runs["out"][label] = (json.loads(r.stdout.strip().splitlines()[-1]), lp)
    if cpu_pods and os.path.exists(DROPIN_CPU):
        d2 = os.path.join(d, "cpu")
        os.makedirs(d2)
        pp2, sp2, pd2 = _dropin_files(d2, spec, ann, now[:cpu_pods], ds[:cpu_pods])
        runs["cpu"] = subprocess.run([DROPIN_CPU, pp2, sp2, pd2, "--threads", str(threads), "--cpu", "--churn", "1"],
                                     capture_output=True, text=True, timeout=900, env=env)
    return runs


def dropin_leg(cd, spec, c, ann, now, ds, threads, dev_index, cpu_pods=0, runs=None):
    """Per-pod cycle of the C++ plugin mirror as the framework drives it (tools/dropin_bench.cpp),
    with its parts, while the controller patches annotations at its own rate (churn x1: every
    (node, metric) re-synced at the policy's periods, metric + node_hot_value per sync) and at 10x
    that rate, plus the frozen snapshot; every pod's chosen node is checked against one engine
    re-uploaded with the churned snapshot (and a pod sample against the oracle).  With cpu_pods > 0
    (the CPU-baseline leg) the same harness drives a CPU plugin that re-parses annotations per
    call (oracle string mode) on the first cpu_pods pods, under the same churn."""
    if runs is None:  # (the harness runs now: this process already holds GPU queues)
        runs = dropin_runs(spec, ann, now, ds, threads, cpu_pods)
    try:
        if runs["err"]:
            return {"error": runs["err"]}
        res, chosen = {}, {}
        for label, (o, lp) in runs["out"].items():
            pnow = runs["now_long"] if label == "nodes_and_time" else now
            ch = chosen[label] = np.array(o.pop("chosen"))
            ref, orc = _replay_chosen(cd, spec, c, dev_index, pnow, ds, lp,
                                      oracle_pods=(0, len(now) // 2, len(now) - 1))
            o["matches_engine_chosen"] = bool(np.array_equal(ch, ref))
            o["matches_oracle_sample"] = orc
            res[label] = o
        rc = runs["cpu"]
    finally:
        shutil.rmtree(runs["dir"], ignore_errors=True)
    runs = res
    out = {}
    main = runs["churn_x1"]
    out["dropin_ms_per_pod"] = main["cycle_ms_median"]
    out["matches_engine_chosen"] = all(r["matches_engine_chosen"] for r in runs.values())
    out["matches_oracle_sample"] = all(r["matches_oracle_sample"] for r in runs.values())
    out["workload"] = (f"{main['nodes']} nodes x {main['pods']} pods (1 ms apart), one scheduling cycle per pod: "
                       f"Filter on every node + Score on every feasible node from {main['threads']} threads + "
                       "selectHost, through include/crane_dyn_plugin.hpp, while the controller patches annotations "
                       "(churn_x1: its rate, each (node, metric) re-synced at the policy's periods; churn_x10: 10x)")
    for label, o in runs.items():
        out[label] = {k: o[k] for k in ("cycle_ms_median", "cycle_ms_p90", "cycle_ms_mean", "cycle_ms_max",
                                        "cycle_ms_max_after_first_change",
                                        "changed_cycle_ms_median", "first_call_ms_median",
                                        "filter_fanout_ms_median", "score_fanout_ms_median", "select_ms_median",
                                        "pool_noop_ms_median", "patches", "simulated_s", "cycles_with_patches",
                                        "tables_built", "full_syncs", "incremental_syncs", "nodes_updated",
                                        "nodes_joined", "nodes_left", "shard_grows", "slowest",
                                        "errors", "sync_ms", "matches_engine_chosen", "matches_oracle_sample")}
    out["how"] = ("each patch publishes a new Node object (informer); the plugin compares every NodeInfo with the "
                  "one it parsed at the cycle's first call, re-parses only the changed nodes (the cycle's callers "
                  "share the parse), writes them into the engine and rebuilds their table rows in one call "
                  "(crane_dyn_update_node_steps); joining nodes take free rows, leaving ones free theirs; "
                  "first_call = that first Filter call; sync_ms = the initial full parse + upload + table; "
                  "pool_noop = the harness's two fan-outs over no-op calls (not part of the cycle); the harness runs "
                  "before the bench process touches the GPU (a scheduler process holds the device alone); checks: "
                  "every pod's chosen node vs one engine re-uploaded with the churned snapshot, 3 pods vs the oracle")
    if rc is not None:
        if rc.returncode != 0:
            out["cpu_same_harness_error"] = rc.stderr[-300:]
        else:
            oc = json.loads(rc.stdout.strip().splitlines()[-1])
            chc = oc.pop("chosen")
            out["cpu_same_harness_ms_per_pod"] = oc["cycle_ms_median"]
            out["cpu_same_harness"] = {
                "pods": oc["pods"], "threads": oc["threads"], "cycle_ms_median": oc["cycle_ms_median"],
                "filter_fanout_ms": oc["filter_fanout_ms_median"], "score_fanout_ms": oc["score_fanout_ms_median"],
                "harness_noop_fanouts_ms": oc["pool_noop_ms_median"], "patches": oc["patches"],
                "how": "same harness, thread pool and churn (x1); Filter / Score re-parse the node's current "
                       "annotations per call like stats.go:51-76 (oracle string mode, oracle/_build/dropin_cpu)"}
            out["cpu_same_harness"]["matches_engine_chosen"] = bool(np.array_equal(np.array(chc),
                                                                                   chosen["churn_x1"][:cpu_pods]))
            out["speedup_vs_cpu_same_harness"] = round(oc["cycle_ms_median"] / main["cycle_ms_median"], 1)
    return out


def controller_leg(cd, O, synth, spec, dev, c, N, B):
    """Controller per-sync hot values (node.go:113-121 over binding.go:81-123) with the
    engine keeping BindingRecords: append one second of bindings (the synthetic log's rate)
    + BindingsGC + K2/K1 + readback, host wall incl. the H2D of the appended slots; and the
    full-replace form (12 B x B uploaded per sync)."""
    eng = cd.Engine(cd.Policy(spec), dev.index)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts)
    gc = max(tr for tr, _ in spec["hotValue"])  # controller.go:57
    eng.binding_records(B, gc)
    eng.add_bindings(c.b_node, c.b_ts)
    rng = np.random.default_rng(5)
    per_s = max(1, B // 600)
    ops, nodes, args = [np.zeros(B, np.uint8)], [c.b_node], [c.b_ts]
    reps = []
    for s in range(1, 7):
        bn = c.b_node[rng.integers(0, B, per_s)]
        bt = np.full(per_s, synth.NOW0 + s, np.int64)
        now_ns = (synth.NOW0 + s) * 10**9
        t1 = time.perf_counter()
        eng.add_bindings(bn, bt)
        eng.gc_bindings(now_ns)
        eng.refresh_hot_values(now_ns, now_ns)
        hv = eng.hot_values()
        if s > 1:
            reps.append(time.perf_counter() - t1)
        ops += [np.zeros(per_s, np.uint8), np.ones(1, np.uint8)]
        nodes += [bn, np.zeros(1, np.int32)]
        args += [bt, np.array([synth.NOW0 + s], np.int64)]
    t1 = time.perf_counter()
    on, ot = O.binding_heap(B, gc, np.concatenate(ops), np.concatenate(nodes), np.concatenate(args))
    _, ohv = O.hot_values(spec, on, ot, N, synth.NOW0 + 6)
    ocpu = time.perf_counter() - t1
    ok = bool(np.array_equal(hv, ohv.astype(np.float64))) and eng.binding_count() == len(on)
    # full replace of the log per sync (upload + K2 + K1 + readback)
    now_ns = int(synth.NOW0_NS)
    full = []
    for r in range(4):
        t1 = time.perf_counter()
        eng.upload_bindings(c.b_node, c.b_ts)
        eng.refresh_hot_values(now_ns, now_ns)
        eng.hot_values()
        if r:
            full.append(time.perf_counter() - t1)
    eng.close()
    return {"workload": f"{B}-entry BindingRecords heap -> {N} node hot values per controller sync",
            "append_sync_ms": round(float(np.median(reps)) * 1e3, 3),
            "append_sync": f"add {per_s} bindings + BindingsGC + K2/K1 + D2H of the hot values, host wall "
                           "(incl. the H2D of the changed log slots)",
            "full_replace_sync_ms": round(float(np.median(full)) * 1e3, 3),
            "full_replace_sync": f"upload all {B} bindings (12 MB H2D) + K2/K1 + D2H, host wall",
            "oracle_cpu_ms": round(ocpu * 1e3, 2),
            "oracle": "C restatement of the container/heap BindingRecords replay + one pass over the heap "
                      "(the reference scans the heap once per node: O(N*B))",
            "matches_oracle": ok}


def launch_ranks(args):
    """`--gpus N > 1` without a launcher: start N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process and return its exit code.  Runs before anything
    touches the GPU (torch.cuda.device_count() does not initialise it on this image)."""
    have = torch.cuda.device_count()
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this host has {have}", file=sys.stderr)
        return 2
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def build_shard(synth, spec, args, world, rank):
    """This rank's node shard, as a deterministic slice of ONE global cluster.
    Config 3 (weak scaling): the global cluster is `world` cells of 100k nodes, each with
    its own 1M-entry binding log; cell r (seed + r) is rank r's shard, so rank r's nodes
    are global [r*100k, (r+1)*100k) for every N.  Config 4 (strong scaling): one 1M-node
    cluster with one 1M-entry binding log (the same arrays at every N); rank r keeps
    shard_range(1M, N, r) and the bindings of its nodes.  Returns (shard, global offset,
    global node count, a function that builds the whole global cluster)."""
    from crane_dyn.shard import shard_range
    cfg = synth.CONFIGS[args.config]
    P, B = cfg["pods"], cfg["bindings"]
    if args.config == 4:
        def whole():
            return synth.make_cluster(spec, cfg["nodes"], P, n_bindings=B, seed=20250215 + 4000)
        full = whole()
        lo, hi = shard_range(cfg["nodes"], world, rank)
        c = full.node_slice(lo, hi) if world > 1 else full
        n_total = cfg["nodes"]
    else:
        def cell(r):
            return synth.make_cluster(spec, cfg["nodes"], P, n_bindings=B, seed=20250215 + args.config * 1000 + r)

        def whole():
            return synth.concat([cell(r) for r in range(world)])
        c = cell(rank)
        lo, n_total = rank * cfg["nodes"], world * cfg["nodes"]
    # the pod batch is the same on every shard (only nodes and bindings are per rank)
    c.now, c.ds = synth.make_pods(P, seed=20250215 + args.config)
    return c, lo, n_total, whole


def keys_one_engine(cd, synth, spec, dev, whole, d_now, d_flags, now_sync):
    """The keys of the batch from ONE engine holding the whole global cluster (its nodes
    and its binding log) on this GPU: what the all-reduced shard keys must equal."""
    g = whole()
    e = cd.Engine(cd.Policy(spec), dev.index)
    gv, gt, _ = g.rows(e.metric_names)
    e.upload_nodes(gv, gt, g.hv, g.hv_ts)
    e.upload_bindings(g.b_node, g.b_ts)
    k = torch.empty(d_now.numel(), dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(dev)
    e.step_keys_async(now_sync, now_sync, d_now, d_flags, k, st.cuda_stream)
    st.synchronize()
    e.close()
    return k, g.n_nodes


def keys_virtual_shards(cd, spec, dev, c, d_now, d_flags, now_sync, ref_keys, S):
    """The batch's keys from S node shards of cluster c on this GPU (ShardedEngine: node_offset,
    each shard's own bindings), max-combined, compared with ref_keys."""
    from crane_dyn.shard import ShardedEngine
    pol = cd.Policy(spec)
    st = torch.cuda.Stream(dev)
    comb = torch.full_like(ref_keys, -1)
    k = torch.empty_like(ref_keys)
    val = ts = None
    for r in range(S):
        se = ShardedEngine(pol, c.n_nodes, S, r, dev.index)
        if val is None:
            val, ts, _ = c.rows(se.engine.metric_names)
        se.upload(val, ts, c.hv, c.hv_ts, c.b_node, c.b_ts)
        se.step_keys(now_sync, now_sync, d_now, d_flags, k, st.cuda_stream)
        st.synchronize()
        comb = torch.maximum(comb, k)
        se.close()
    return bool(torch.equal(comb, ref_keys))


def oracle_sample(spec, g, names, pod_now, now, keys, n=64):
    """The batch's keys against the CPU oracle (oracle/crane_oracle.c, a checker: after the timed
    region) on an n-pod sample — evenly spread pods plus the first DaemonSet ones — with the hot
    values the controller computes from the binding log at `now` (O.hot_values, binding.go:81-97)
    stamped `now`, as the step stamps them: chosen node and score per sampled pod."""
    from oracle import oracle as O
    P = len(pod_now)
    smp = np.unique(np.concatenate([np.linspace(0, P - 1, n - 8).astype(np.int64), np.flatnonzero(g.ds)[:8]]))
    _, hv = O.hot_values(spec, g.b_node, g.b_ts, g.n_nodes, int(now) // 10**9)
    val, ts, ok = g.rows(names)
    ff, sc, och = O.eval_soa(spec, names, ok, val, np.where(ok == 1, ts, 0), np.ones(g.n_nodes, np.uint8),
                             hv.astype(np.float64), np.full(g.n_nodes, int(now), np.int64), pod_now[smp], g.ds[smp],
                             threads=16, want_matrix=g.n_nodes * len(smp) <= (1 << 24))
    knode = np.where(keys[smp] < 0, -1, 0xFFFFFFFF - (keys[smp] & 0xFFFFFFFF))
    kscore = np.where(keys[smp] < 0, -1, keys[smp] >> 32)
    ok_node = bool(np.array_equal(knode, och))
    ok_score = None
    if sc is not None:
        feas = (ff < 0) | (g.ds[smp][:, None] != 0)
        best = np.where(feas.any(1), np.where(feas, sc, -1).max(1), -1)
        ok_score = bool(np.array_equal(kscore, best))
    return {"oracle_sample": ok_node and ok_score is not False, "oracle_pods": int(len(smp)),
            "oracle_scores_checked": ok_score is not None}


def k2_read(spec, b_ts, now_ns):
    """The bindings K2 reads, as the engine decides (engine option k2_sorted, default on): a
    log in time order is read from the first binding inside the widest window on, node ids
    only (4 B each: the window rank comes from the position); otherwise every binding's node
    id and stamp (12 B)."""
    B = len(b_ts)
    if B and np.all(b_ts[1:] >= b_ts[:-1]) and spec["hotValue"]:
        cmin = min(now_ns // 10**9 - tr // 10**9 for tr, _ in spec["hotValue"])
        first = int(np.searchsorted(b_ts, cmin, side="right"))
        return {"first": first, "read": B - first, "bytes": 4 * (B - first),
                "what": f"node ids of the {B - first} bindings inside the widest window read (time-ordered log)"}
    return {"first": 0, "read": B, "bytes": 12 * B, "what": "bindings read (node id + stamp)"}


def batch_times(c, args):
    """The timed batches' times (bench realism): batch i is scheduled at now_i = now0 + (i % C) x the
    batch's span (the P pods' own spread, 10 s at config 3), its pods at their times shifted by the
    same amount, so the hot-value cutoffs move every batch and the K2 suffix search reruns.  C
    (--now-cycle, 6 = one minute of pod time) bounds the drift: the synthetic snapshot and binding
    log are not re-synced between batches, and further out every 5-minute metric would go stale.
    Returns (now_ns per cycle position, pod times per cycle position, span)."""
    step = int(c.now[1] - c.now[0]) if len(c.now) > 1 else 10**9
    span = int(c.now[-1] - c.now[0]) + step
    C = max(1, args.now_cycle)
    now0 = int(c.now[0])
    return [now0 + j * span for j in range(C)], [c.now + j * span for j in range(C)], span


def measure_ranks(cd, synth, spec, args, world, rank, local, dev):
    """One rank per GPU (this process's GPU `local`): its node shard on K engines, batches in flight on
    K streams; N > 1: one RCCL max all-reduce of a group of batches' keys (torch.distributed)."""
    coll = world > 1 or args.rehearse_collective
    strong = args.config == 4
    c, node_lo, n_total, whole = build_shard(synth, spec, args, world, rank)
    N, P = c.n_nodes, len(c.now)
    K = max(1, args.inflight)
    engs = [cd.Engine(cd.Policy(spec), local) for _ in range(K)]
    eng = engs[0]
    val, ts, _ = c.rows(eng.metric_names)
    for e in engs:
        e.upload_nodes(val, ts, c.hv, c.hv_ts, node_offset=node_lo)
        e.upload_bindings(c.b_node, c.b_ts)
    nows, pods, span = batch_times(c, args)
    C = len(nows)
    d_now = [torch.from_numpy(p).to(dev) for p in pods]
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys_k = [torch.empty(P, dtype=torch.int64, device=dev) for _ in range(K)]
    # dedicated streams: the default stream's handle is 0, which the C ABI reads as "engine stream"
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    torch.cuda.set_stream(streams[0])
    sh_k = [s_.cuda_stream for s_ in streams]
    # N > 1: one RCCL max all-reduce per group of G batches over their keys [G][P], on its own
    # stream after the group's K streams; two key buffers alternate so a group's batches never
    # overwrite keys a collective still reads
    G = max(K, args.ar_group or 16 * K) // K * K  # batches per collective, a multiple of K
    if coll:
        kbufs = [torch.empty((G, P), dtype=torch.int64, device=dev) for _ in range(2)]
        cstream = torch.cuda.Stream(dev)
        ar_done = [None, None]
        ev_s = [torch.cuda.Event() for _ in range(K)]  # (reused: record() re-arms an event)
        ev_ar = [torch.cuda.Event(), torch.cuda.Event()]

    def collect(b, nb):
        for jj in range(min(nb, K)):
            ev_s[jj].record(streams[jj])
            cstream.wait_event(ev_s[jj])
        with torch.cuda.stream(cstream):
            dist.all_reduce(kbufs[b][:nb], op=dist.ReduceOp.MAX)  # RCCL over xGMI
        ev_ar[b].record(cstream)
        ar_done[b] = ev_ar[b]

    # the step calls bound once to their engine, stream, pod batch and key buffer
    step_own = [[engs[j].step_keys_fn(d_now[t], d_flags, d_keys_k[j], sh_k[j]) for t in range(C)] for j in range(K)]
    step_grp = ([[[engs[r % K].step_keys_fn(d_now[t], d_flags, kbufs[b][r], sh_k[r % K]) for t in range(C)]
                  for r in range(G)] for b in range(2)] if coll else None)

    def step(collective=True, i=0):
        j, t = i % K, i % C
        if coll and collective:
            b, row = (i // G) % 2, i % G
            if row < K and ar_done[b] is not None:  # this buffer's previous collective has read it
                streams[j].wait_event(ar_done[b])
            step_grp[b][row][t](nows[t], nows[t])
            if row == G - 1:
                collect(b, G)
        else:
            step_own[j][t](nows[t], nows[t])

    def flush(n_steps):  # the last, partial group's collective
        if coll and n_steps % G:
            collect((n_steps // G) % 2, n_steps % G)

    for i in range(args.warmup):
        step(i=i)
    flush(args.warmup)
    if coll:
        # RCCL's first call at a given size sets that size up: untimed, once at every size the
        # timed region reduces, so no setup lands in the timing
        for b in range(2):
            for nb in sorted({G, args.steps % G or G}):
                collect(b, nb)
        ar_done[0] = ar_done[1] = None  # the timed groups start from fresh buffers
    torch.cuda.synchronize(dev)
    if coll:
        dist.barrier()
    cpu0 = task_cpu()
    t0 = time.perf_counter()
    tc0 = time.thread_time()
    for i in range(args.steps):
        step(i=i)
    flush(args.steps)
    t_enq = time.perf_counter() - t0
    tc_enq = time.thread_time() - tc0
    torch.cuda.synchronize(dev)
    if coll:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    host = host_threads(cpu0, task_cpu(), t_enq, tc_enq, elapsed, args.steps)
    if coll:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    t_last = (args.steps - 1) % C
    if coll:  # the last group's keys (all-reduced over the ranks)
        last = kbufs[((args.steps - 1) // G) % 2]
        d_keys = last[(args.steps - 1) % G]
        keys_agree = True
    else:
        d_keys = d_keys_k[(args.steps - 1) % K]
        keys_agree = all(torch.equal(d_keys, k) for k in d_keys_k) if C == 1 else None
    keys = d_keys.cpu().numpy()
    keys_match, keys_match_how = None, "single rank: no combine step"
    if coll:
        if rank == 0:
            ref_k, n_glob = keys_one_engine(cd, synth, spec, dev, whole, d_now[t_last], d_flags, nows[t_last])
            assert n_glob == n_total
            keys_match = bool(torch.equal(ref_k, d_keys))
        dist.barrier()
        keys_match_how = ("the last batch's all-reduced keys [P] == one engine holding the whole "
                          f"{n_total}-node global cluster and its binding log, same pods")
    elif world == 1 and strong:
        # config 4 on one GPU: the 8-GPU layout's combine rehearsed on this GPU
        keys_match = keys_virtual_shards(cd, spec, dev, c, d_now[t_last], d_flags, nows[t_last], d_keys, 8)
        keys_match_how = ("8 node shards of the 1M-node cluster (125k nodes each, node_offset, each with its own "
                          "nodes' bindings) on this GPU, their keys max-combined (the all-reduce's operation) == "
                          "the one-engine keys of the last timed batch")
    # one batch's latency: the same step with nothing else in flight (outside the timed region)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    nl = max(10, args.steps // 4)
    for i in range(nl):
        step(collective=False, i=i * K)  # (engine 0 only: each batch waits for the previous one on its stream)
        if coll:
            with torch.cuda.stream(streams[0]):
                dist.all_reduce(d_keys_k[0], op=dist.ReduceOp.MAX)
    torch.cuda.synchronize(dev)
    batch_latency_ms = (time.perf_counter() - t1) * 1e3 / nl
    kt = kernel_times(eng, lambda: step(collective=False), args.steps)
    ar_ms = None
    if coll:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        with torch.cuda.stream(streams[0]):
            for _ in range(10):
                dist.all_reduce(d_keys, op=dist.ReduceOp.MAX)
        e1.record(streams[0])
        torch.cuda.synchronize(dev)
        ar_ms = e0.elapsed_time(e1) / 10
    m = dict(c=c, N=N, P=P, n_total=n_total, val=val, ts=ts, eng=eng, ms_step=elapsed * 1e3 / args.steps,
             keys=keys, keys_agree=keys_agree, keys_match=keys_match, keys_match_how=keys_match_how, host=host,
             batch_latency_ms=batch_latency_ms, kt=kt, ar_ms=ar_ms, K=K, nows=nows, span=span, stream=streams[0],
             how=("K engines (own copy of the shard's nodes, binding log, scratch) on K HIP streams, batch i on "
                  "engine i % K; every batch runs the whole step" +
                  (f"; one RCCL max all-reduce (torch.distributed, one process per GPU) per group of {G} batches' "
                   f"keys [{G}][P] on its own stream" if coll else "")),
             engine_path="ranks" + (" (torch.distributed RCCL)" if coll else ""), n_gpus=world)
    m["close"] = lambda: [e.close() for e in engs]
    return m


def measure_group(cd, synth, spec, args, n_dev, dev):
    """One process driving n_dev GPUs through the C ABI group (crane_dyn_group_*, group.cpp): the
    global cluster's node shards over the devices, K batches in flight (the group's slots), each
    batch = every device's shard step + the in-library RCCL max all-reduce of the keys (n_dev > 1;
    with one device there is nothing to combine)."""
    from crane_dyn.shard import shard_range
    strong = args.config == 4
    cfg = synth.CONFIGS[args.config]
    P, B = cfg["pods"], cfg["bindings"]
    if strong:
        g_all = synth.make_cluster(spec, cfg["nodes"], P, n_bindings=B, seed=20250215 + 4000)
    else:
        cells = [synth.make_cluster(spec, cfg["nodes"], P, n_bindings=B, seed=20250215 + args.config * 1000 + r)
                 for r in range(n_dev)]
        g_all = synth.concat(cells) if n_dev > 1 else cells[0]
    g_all.now, g_all.ds = synth.make_pods(P, seed=20250215 + args.config)
    n_total = g_all.n_nodes
    lo0, hi0 = shard_range(n_total, n_dev, 0)
    c = g_all if n_dev == 1 else g_all.node_slice(lo0, hi0)  # device 0's shard (per-kernel rooflines)
    c.now, c.ds = g_all.now, g_all.ds
    K = max(1, args.inflight)
    grp = cd.Group(cd.Policy(spec), devices=list(range(n_dev)), depth=K)
    grp.set_option("collective", args.group_collective)
    grp.set_option("threads", args.group_threads)
    coll_on = args.group_collective == 2 or (args.group_collective == 1 and n_dev > 1)
    dispatch = args.group_dispatch if args.group_dispatch >= 0 else 1
    grp.set_option("dispatch", dispatch)
    for o in args.opt:  # engine options (name=value) on every slot's engines
        k, v = o.split("=")
        grp.set_option(k, int(v))
    val_all, ts_all, _ = g_all.rows(grp.metric_names)
    grp.upload_nodes(val_all, ts_all, g_all.hv, g_all.hv_ts)
    grp.upload_bindings(g_all.b_node, g_all.b_ts)
    nows, pods, span = batch_times(g_all, args)
    C = len(nows)
    devs = [torch.device("cuda", d) for d in range(n_dev)]
    d_now = [[torch.from_numpy(p).to(dv) for dv in devs] for p in pods]
    d_flags = [torch.from_numpy(g_all.ds).to(dv) for dv in devs]
    # two key buffers per slot, alternating: a slot's step leaves its last kernel (K3s) to the slot's
    # next step (engine option step_defer, set by the group on its queues), which must not reset
    # keys it still writes
    d_keys = [[torch.empty(P, dtype=torch.int64, device=dv) for dv in devs] for _ in range(2 * K)]
    seq = [0]  # batches enqueued on the group so far: batch b runs on slot b % K
    recent = []  # (keys getter, cycle position) of the latest batches, newest last
    if not coll_on:
        # one batch per call (crane_dyn_group_step_keys_async)
        fns = [[grp.step_keys_fn(d_now[t], d_flags, d_keys[s]) for t in range(C)] for s in range(2 * K)]
        G = 1

        def step(i):
            t = i % C
            s_ = seq[0] % (2 * K)
            fns[s_][t](nows[t], nows[t])
            recent.append((lambda s_=s_: d_keys[s_][0], t))
            del recent[:-2]
            seq[0] += 1
    else:
        # the collective: windows of G batches per call (crane_dyn_group_step_keys_batch), ONE
        # all-reduce of a window's keys [G][P] per device, two key buffers alternating
        G = max(1, args.ar_group or min(args.steps, 64))
        gdn = {}  # (first cycle position, rows) -> per-device pod times [rows][P]
        gfl = [torch.from_numpy(np.tile(g_all.ds, (G, 1))).to(dv) for dv in devs]
        gkeys = [[torch.empty((G, P), dtype=torch.int64, device=dv) for dv in devs] for _ in range(2)]
        gfns = {}
        win = [0]

        def window(i0, rows):
            key = (i0 % C, rows)
            if key not in gdn:
                gdn[key] = [torch.from_numpy(np.stack([pods[(i0 + j) % C] for j in range(rows)])).to(dv) for dv in devs]
            b = win[0] % 2
            fk = (key, b)
            if fk not in gfns:
                gfns[fk] = grp.step_keys_batch_fn(gdn[key], [f[:rows] for f in gfl], [k[:rows] for k in gkeys[b]])
            ts_ = [nows[(i0 + j) % C] for j in range(rows)]
            gfns[fk](ts_, ts_)
            for j in range(max(0, rows - 2), rows):
                recent.append((lambda b=b, j=j: gkeys[b][0][j], (i0 + j) % C))
            del recent[:-2]
            seq[0] += rows
            win[0] += 1

        def step(i):  # (a one-batch window: warmup and the latency loop)
            window(i, 1)

    def sync_all():
        grp.sync()
        for dv in devs:
            torch.cuda.synchronize(dv)

    dispatch_note = None
    try:
        step(0)  # (the first batch makes the dispatch queues)
    except cd.CraneError as e:
        if args.group_dispatch >= 0:
            raise
        # auto: a box whose runtime refuses the queues keeps HIP launches, and the line says so
        dispatch_note = f"dispatch queues unavailable ({e}); HIP launches on the slots' streams"
        dispatch = 0
        grp.set_option("dispatch", 0)
        step(0)
    for i in range(1, args.warmup):
        step(i)
    if coll_on:  # (every window shape of the timed region once, untimed: RCCL sets up per size)
        for rows in sorted({G, args.steps % G or G}):
            window(0, rows)
            window(0, rows)
    sync_all()
    cpu0 = task_cpu()
    t0 = time.perf_counter()
    tc0 = time.thread_time()
    if coll_on:
        for i0 in range(0, args.steps, G):
            window(i0, min(G, args.steps - i0))
    else:
        for i in range(args.steps):
            step(i)
    t_enq = time.perf_counter() - t0
    tc_enq = time.thread_time() - tc0
    grp.sync()
    elapsed = time.perf_counter() - t0
    host = host_threads(cpu0, task_cpu(), t_enq, tc_enq, elapsed, args.steps)
    t_last = (args.steps - 1) % C
    last_get, _ = recent[-1]
    keys = last_get().cpu().numpy()
    if n_dev > 1:  # every device holds the all-reduced keys
        keys_agree = True
        if coll_on:
            b_last = (win[0] - 1) % 2
            row = (args.steps - 1) % G
            keys_agree = all(torch.equal(gkeys[b_last][0][row].cpu(), gkeys[b_last][d][row].cpu())
                             for d in range(1, n_dev))
    else:
        keys_agree = None
    # the timed path pinned at full size: the last timed batch and the one before it (another slot,
    # another `now`: the cutoffs moved between them) against one engine over the whole cluster on a
    # HIP stream and against the CPU oracle on a pod sample (checker only, after the timed region)
    pinned = []
    for get_, t_ in reversed(recent):
        ref_k, _ = keys_one_engine(cd, synth, spec, devs[0], lambda: g_all, d_now[t_][0], d_flags[0], nows[t_])
        got = get_().cpu().numpy()
        pinned.append({"now_ns": int(nows[t_]), "stream": bool(np.array_equal(ref_k.cpu().numpy(), got)),
                       **oracle_sample(spec, g_all, grp.metric_names, pods[t_], nows[t_], got)})
    keys_match, keys_match_how = None, "one device: no combine step"
    if n_dev > 1:
        keys_match = pinned[0]["stream"] and bool(keys_agree)
        keys_match_how = ("the last batch's all-reduced keys on every device == one engine holding the whole "
                          f"{n_total}-node global cluster and its binding log, same pods")
    elif strong:
        keys_match = keys_virtual_shards(cd, spec, dev, c, d_now[t_last][0], d_flags[0], nows[t_last],
                                         torch.from_numpy(keys).to(dev), 8)
        keys_match_how = ("8 node shards of the 1M-node cluster (125k nodes each, node_offset, each with its own "
                          "nodes' bindings) on this GPU, their keys max-combined (the all-reduce's operation) == "
                          "the group's keys of the last timed batch")
    sync_all()
    nl = max(10, args.steps // 4)
    t1 = time.perf_counter()
    for i in range(nl):
        step(i)  # (with the collective: a one-batch window and its all-reduce)
        grp.sync()
    batch_latency_ms = (time.perf_counter() - t1) * 1e3 / nl
    # per-kernel durations: shard 0's engine of slot 0 stepping the same batch on its own stream
    coll = args.group_collective == 2 or (args.group_collective == 1 and n_dev > 1)
    workers = args.group_threads == 1 or (args.group_threads == -1 and n_dev > 1)
    eng = grp.engine(0, 0)
    st0 = torch.cuda.Stream(devs[0])
    k0 = torch.empty(P, dtype=torch.int64, device=devs[0])
    kcyc = [0]

    def kstep():  # the timed batches' times in turn (the delta form's changed bindings vary with them)
        t = kcyc[0] % len(nows)
        kcyc[0] += 1
        eng.step_keys_async(nows[t], nows[t], d_now[t][0], d_flags[0], k0, st0.cuda_stream)

    kt = kernel_times(eng, kstep, max(args.steps, 2 * len(nows)))
    val, ts, _ = c.rows(grp.metric_names)
    m = dict(c=c, N=c.n_nodes, P=P, n_total=n_total, val=val, ts=ts, eng=eng, ms_step=elapsed * 1e3 / args.steps,
             keys=keys, keys_agree=keys_agree, keys_match=keys_match, keys_match_how=keys_match_how, host=host,
             pinned=pinned, batch_latency_ms=batch_latency_ms, kt=kt, ar_ms=None, K=K, nows=nows, span=span, stream=st0,
             how=(f"one process, crane_dyn_group over {n_dev} device(s) (C ABI, group.cpp): {K} batch slots, each "
                  "with an engine per device (the slots of a device share one copy of its shard's nodes and log) "
                  "on its own stream or dispatch queue, batch i on slot i % K; every batch runs the whole shard "
                  "step on every device" +
                  (f"; windows of {G} batches (crane_dyn_group_step_keys_batch), then ONE in-place RCCL "
                   f"ncclAllReduce(int64, max) of a window's keys [{G}][P] per device on a collective stream "
                   "ordered after the dispatch queues (ncclCommInitAll communicators)" if coll else "") +
                  ("; enqueued by one worker thread per device" if workers else "; enqueued by the caller's thread") +
                  ("; the step's kernels written as AQL packets to one user-mode queue per slot (crane_queue: "
                   "~0.3 us per kernel instead of a HIP launch's 2.6-3.7 us)" if dispatch else
                   "; the step's kernels launched through HIP on the slots' streams")),
             engine_path=("group (C ABI, in-library RCCL" + (", rehearsed on one device)" if n_dev == 1 else ")")
                          if coll else "group (C ABI, one device)") + (", dispatch queues" if dispatch else ""),
             dispatch_note=dispatch_note, n_gpus=n_dev)
    m["close"] = lambda: grp.close()
    return m


def main():
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if launched and world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if not launched and args.gpus > 1:
        have = torch.cuda.device_count()  # (does not initialise the GPU on this image)
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this host has {have}", file=sys.stderr)
            sys.exit(2)
        if args.engine == "ranks":
            sys.exit(launch_ranks(args))
    group = args.engine == "group" and not args.rehearse_collective
    if group and launched and world > 1:
        # the group drives every device from rank 0's process; the launcher's other ranks only
        # wait (CPU barrier), touching no GPU
        dist.init_process_group("gloo")
        if rank != 0:
            dist.barrier()
            dist.destroy_process_group()
            return
    elif not group and (world > 1 or args.rehearse_collective):
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import crane_dyn as cd
    from crane_dyn import synth

    spec = cd.default_policy_spec()
    # the drop-in harness runs first, while this process holds no GPU queue (dropin_runs); its
    # snapshot is the config-3 cell measure_group builds (same seeds), checked there
    early = None
    if (args.leg == "all" and group and args.gpus == 1 and not args.no_extras and not args.no_cpu_baseline
            and args.config == 3 and rank == 0):
        cfg = synth.CONFIGS[3]
        c0 = synth.make_cluster(spec, cfg["nodes"], cfg["pods"], n_bindings=cfg["bindings"], seed=20250215 + 3000)
        c0.now, c0.ds = synth.make_pods(cfg["pods"], seed=20250215 + 3)
        ann0 = c0.annotations()
        early = {"c": c0, "ann": ann0,
                 "runs": dropin_runs(spec, ann0, c0.now[:256], c0.ds[:256], args.cpu_threads, cpu_pods=4)}
    args.early = early

    dev = torch.device("cuda", local if not group else 0)
    torch.cuda.set_device(dev)
    shash = src_hash()
    if args.leg == "cold":
        pmc_c, pmc_cs = pmc_summary("cold", shash)
        out = cold_leg(cd, synth, spec, dev, reps=max(2, args.steps), pmc=pmc_c, pmc_src=pmc_cs, opts=args.opt)
        print(json.dumps({"leg": "cold", "src_hash": shash, "lib_hash": lib_hash(), **out}), flush=True)
        return
    if args.leg != "all":
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        cid = 2 if args.leg == "matrix2" else 3
        cm = synth.make_cluster(spec, synth.CONFIGS[cid]["nodes"], synth.CONFIGS[cid]["pods"], seed=20250215 + cid)
        names = cd.Engine(cd.Policy(spec), local).metric_names
        vm, tm, _ = cm.rows(names)
        pmc_m, _ = pmc_summary("2" if cid == 2 else "3m", shash)
        out = matrix_leg(cd, spec, dev, stream, f"config{cid} full matrices", vm, tm, cm.hv, cm.hv_ts, cm.now, cm.ds,
                         args.steps, pmc_m)
        print(json.dumps({"leg": args.leg, "src_hash": shash, "lib_hash": lib_hash(), **out}), flush=True)
        return

    if group:
        m = measure_group(cd, synth, spec, args, args.gpus, dev)
        n_gpus, solo = args.gpus, True
    else:
        m = measure_ranks(cd, synth, spec, args, world, rank, local, dev)
        n_gpus, solo = world, world == 1
    finish(cd, synth, spec, args, m, n_gpus, rank, solo, dev, shash)
    m["close"]()
    if dist.is_initialized():
        if group:
            dist.barrier()  # (the other ranks are waiting here)
        dist.destroy_process_group()


def finish(cd, synth, spec, args, m, n_gpus, rank, solo, dev, shash):
    """Rooflines, the extra legs (one GPU) and the JSON line (rank 0)."""
    strong = args.config == 4
    c, N, P, n_total, val, ts, eng, kt = m["c"], m["N"], m["P"], m["n_total"], m["val"], m["ts"], m["eng"], m["kt"]
    B = len(c.b_node)
    ms_step = m["ms_step"]
    stream = m["stream"]
    local = dev.index
    pairs_per_s = P * n_total / (ms_step / 1e3)
    placements = P / (ms_step / 1e3)
    now_sync = m["nows"][0]

    # Rooflines per kernel: ALGORITHMIC bytes per launch / the kernel's
    # mean dispatch-stamped duration.  K3s re-reads L2-resident step records: not HBM-priced.
    M, W = len(eng.metric_names), len(spec["hotValue"])
    kb = k2_read(spec, c.b_ts, now_sync)
    cut = np.sort(np.array([now_sync // 10**9 - tr // 10**9 for tr, _ in spec["hotValue"]], np.int64))
    jr = (c.b_ts[:, None] > cut[None, :]).sum(1)
    okb = (jr > 0) & (c.b_node >= 0) & (c.b_node < N)
    # dedupe-form K2: one 4-byte entry per distinct (2048-binding region, node, window rank),
    # a (count, offset) word per (node block, region); the node pass reads both.  Regions
    # start at the first binding K2 reads (a time-ordered log: the widest window's suffix)
    reg = (np.arange(B, dtype=np.int64) - kb["first"]) // 2048
    E = int(np.unique((reg[okb] * (N + 1) + c.b_node[okb]) * 8 + jr[okb] - 1).size) if B else 0
    co_b = 4 * (-(-N // 256)) * (-(-kb["read"] // 2048))
    k3p_b = P * (8 + 1 + 4 + 8 + 8)
    k2d_b = kb["bytes"] + E * 4 + co_b
    dl = delta_changed(spec, c.b_ts, m["nows"])
    alg = {
        "k2x_dedupe": (k2d_b, kb["what"] + " + distinct (region, node, bucket) entries + count/offset written"),
        "k2x_dedupe+k3p_pods": (k2d_b + k3p_b, kb["what"] + " + distinct entries + count/offset written; pod now + "
                                               "flag read, partition + keys written"),
        "k1_node_pass+k3a_steps": (N * (16 * M + 8) + E * 4 + co_b,
                                   "SoA (value, ts) read + hot value written + K2 entries and count/offset read"),
        "k1_stream_steps": (N * (16 * M + 8 + 4 * W), "SoA (value, ts) read + hot value written + window counts read"),
        "k3p_pods": (k3p_b, "pod now + flag read, partition + keys written"),
        "k2_delta+k3p_pods": (12 * dl["mean"] + k3p_b,
                              "per changed binding (window rank differs from the anchor refresh's): node id read "
                              "+ its -1 / +1 adjustments written (12 B, mean over the timed batches' times); pod now "
                              "+ flag read, partition + keys written"),
    }
    pmc, pmc_src = pmc_summary(args.config, shash)
    roofs = {}
    for name, t in kt.items():
        if name in alg and t > 0:
            roofs[name] = roof(alg[name][0], t, alg[name][1], pmc_traffic(pmc, name))
    dom = max(kt, key=kt.get) if kt else None
    rname = dom if dom in roofs else (max(roofs, key=lambda k: kt[k]) if roofs else None)
    roofline = dict(roofs[rname], kernel=rname, dominant_kernel=dom) if rname else None
    if roofline is not None:
        roofline["traffic_source"] = pmc_src if roofline.get("traffic") is not None else None
        if rname != dom:
            roofline["note"] = (f"the longest kernel ({dom}, {kt[dom]:.4f} ms) re-reads L2-resident step records "
                                "per pod tile and has no HBM roofline; this is the longest HBM-priced kernel")

    extras = {}
    one = solo and n_gpus == 1 and rank == 0
    if one and not args.no_extras:
        # BASELINE config 2 and the per-pair rate at config 3: every pair's result in HBM
        c2 = synth.make_cluster(spec, synth.CONFIGS[2]["nodes"], synth.CONFIGS[2]["pods"], seed=20250215 + 2)
        v2, t2, _ = c2.rows(eng.metric_names)
        pmc2, _ = pmc_summary("2", shash)
        extras["matrix_config2"] = matrix_leg(
            cd, spec, dev, stream, "config2: 5000 nodes x 1000 pods, full first-fail + score matrices + chosen node",
            v2, t2, c2.hv, c2.hv_ts, c2.now, c2.ds, max(args.steps, 20), pmc2)
        if args.config == 3:
            extras["select_config3"] = select_leg(cd, spec, dev, stream, val, ts, c.hv, c.hv_ts, c.now, c.ds)
            extras["matrix_config3"] = matrix_leg(
                cd, spec, dev, stream, "config3 nodes/pods (100000 x 10000), node_hot_value annotations: full "
                "first-fail + score matrices (2 x 1 GB int8) + chosen node", val, ts, c.hv, c.hv_ts, c.now, c.ds, 10,
                pmc_summary("3m", shash)[0])

    roofline_cold = None
    if one and not args.no_extras and not args.no_cold:
        pmc_c, pmc_cs = pmc_summary("cold", shash)
        roofline_cold = cold_leg(cd, synth, spec, dev, pmc=pmc_c, pmc_src=pmc_cs)

    greedy = None
    if one and not args.no_greedy and not args.no_extras:
        # BASELINE config 5: 100k nodes x 50k pods placed sequentially, each binding
        # raising the chosen node's hot value before the next pod (one GPU).
        g5 = synth.CONFIGS[5]
        cg = synth.make_cluster(spec, g5["nodes"], g5["pods"], n_bindings=g5["bindings"], seed=20255215)
        geng = cd.Engine(cd.Policy(spec), local)
        gv, gt, _ = cg.rows(geng.metric_names)
        geng.upload_nodes(gv, gt, cg.hv, cg.hv_ts)
        geng.upload_bindings(cg.b_node, cg.b_ts)
        geng.greedy(g5["pods"], now_sync, cg.ds)  # warmup
        gt_ms = []
        for _ in range(3):
            t1 = time.perf_counter()
            gch = geng.greedy(g5["pods"], now_sync, cg.ds)
            gt_ms.append((time.perf_counter() - t1) * 1e3)
        gms = float(np.median(gt_ms))
        greedy = {"workload": f"config5: {g5['nodes']} nodes x {g5['pods']} pods sequential greedy, one now, "
                              f"{g5['bindings']}-entry binding log", "ms": round(gms, 3),
                  "placements_per_s": round(g5["pods"] / (gms * 1e-3), 1),
                  "full_rescan_equiv_evals_per_s": round(g5["pods"] * g5["nodes"] / (gms * 1e-3), 1),
                  "placed": int((gch >= 0).sum()), "timing": "host wall incl. K2+K1+prep+H2D/D2H of pods"}
        geng.close()

    cpu = None
    host_parse = None
    if one and not args.no_cpu_baseline and args.config == 3:
        # (the headline configuration only: config 4's 1M-node annotation strings alone take minutes to build)
        from oracle import oracle as O
        early = getattr(args, "early", None)
        same = (early is not None and early["c"].n_nodes == c.n_nodes and np.array_equal(early["c"].hv, c.hv)
                and np.array_equal(early["c"].now, c.now) and np.array_equal(early["c"].b_node, c.b_node))
        ann = early["ann"] if same else c.annotations()
        if early is not None and not same:
            shutil.rmtree(early["runs"]["dir"], ignore_errors=True)
        ncpu = effective_cpus()
        legs = {}
        for label, th in (("threads_16", args.cpu_threads), ("threads_all", ncpu)):
            cp = min(P, max(64, args.cpu_pods * th // args.cpu_threads))
            t1 = time.perf_counter()
            O.eval_strings(spec, ann, c.now[:cp], c.ds[:cp], threads=th, want_matrix=False)
            dt = time.perf_counter() - t1
            legs[label] = {"value": round(cp * N / dt, 1), "cores": th,
                           "sample": f"{cp} pods x {N} nodes, {th} threads, {dt:.1f}s"}
        okr = c.rows(eng.metric_names)[2]
        cp = min(P, args.cpu_pods)
        t1 = time.perf_counter()
        O.eval_soa(spec, eng.metric_names, okr, val, ts, np.ones(N, np.uint8), c.hv, c.hv_ts, c.now[:cp], c.ds[:cp],
                   threads=args.cpu_threads, want_matrix=False)
        dts = time.perf_counter() - t1
        # the headline's unit: a placement evaluates the pod against every node of the shard
        cpu = {"value": round(legs["threads_16"]["value"] / N, 2), "unit": "placements/s",
               "evals_per_s": legs["threads_16"]["value"], "cores": args.cpu_threads,
               "kind": "port",
               "sample": f"{legs['threads_16']['sample']}; string mode: every Filter/Score call re-parses its "
                         "annotations like stats.go:51-76 (oracle/crane_oracle.c)",
               "cpu_model": cpu_model(), "nproc": os.cpu_count(), "effective_cpus": ncpu,
               "all_available_cpus": dict(legs["threads_all"], note=f"every CPU this process may use ({ncpu} of "
                                                                     f"nproc {os.cpu_count()}: affinity mask / cgroup "
                                                                     "quota)"),
               "note": f"placements/s = evals/s / {N} nodes (every node's Filter + Score per pod). "
                       "C restatement, not the Go plugin (no Go toolchain, SURVEY 8c); it resolves the fixed-offset "
                       "zone once instead of utils.GetLocation's time.LoadLocation on every call (utils.go:35-45), "
                       "so it is a stronger baseline than the reference",
               "soa_mode": {"value": round(cp * N / dts, 1), "unit": "pod-node evals/s", "cores": args.cpu_threads,
                            "sample": f"{cp} pods x {N} nodes, pre-parsed SoA, {dts:.1f}s"}}
        # the once-per-sync host parse of the same snapshot's annotation
        # strings into the SoA the engine uploads (crane_parse_annotations, C++ threads)
        snap = cd.SnapshotStrings(eng.metric_names, ann)
        host_parse = {"strings": len(snap), "nodes": N}
        for label, th in (("threads_16", args.cpu_threads), ("threads_all", ncpu)):
            snap.parse(synth.SHANGHAI, th)
            reps = []
            for _ in range(3):
                t1 = time.perf_counter()
                snap.parse(synth.SHANGHAI, th)
                reps.append(time.perf_counter() - t1)
            dtp = float(np.median(reps))
            host_parse[label] = {"ms_per_sync": round(dtp * 1e3, 2), "strings_per_s": round(len(snap) / dtp, 1),
                                 "threads": th}
        pv, pt, _, _ = snap.soa()
        okm = okr.astype(bool)
        host_parse["matches_generator_soa"] = bool(np.array_equal(pt[okm], ts[okm]) and np.array_equal(pv[okm],
                                                                                                       val[okm]))
        if not args.no_extras and args.config == 3:
            # the drop-in plugin cycle under annotation churn, and the
            # controller's hot-value sync
            extras["dropin"] = dropin_leg(cd, spec, c, ann, c.now[:256], c.ds[:256], args.cpu_threads, local,
                                          cpu_pods=4, runs=early["runs"] if same else None)
            extras["controller_hot_values"] = controller_leg(cd, O, synth, spec, dev, c, N, B)

    if rank == 0:
        keys = m["keys"]
        line = {
            "metric": "placements/sec",
            "value": round(placements, 1),
            "unit": "placements/s",
            "value_kind": ("pods placed per second, measured: each timed step schedules a batch of "
                           f"{P} pods (Filter + Score of every pod on every node, hot values from the binding log, "
                           "the best feasible node per pod); the per-pair rate with every pair's result written to "
                           "HBM is matrix_config3.evals_per_s"),
            "pairs_decided_per_s": round(pairs_per_s, 1),
            "pairs_decided_note": ("P x nodes_total / step time: every (pod, node) pair's answer is decided exactly, "
                                   "but the step path evaluates a node per pod only where one of its expiries falls "
                                   "inside the batch (DESIGN.md 4.4): a full-rescan equivalent, not an evaluation "
                                   "count; with node shards over N GPUs (weak scaling) it grows with the cluster"),
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": (f"config{args.config}: {n_total} nodes ({N} per GPU) x {P} pods, 6 metrics, "
                                    + (f"hot values from one {synth.CONFIGS[4]['bindings']}-entry binding log over "
                                       "all nodes (each GPU holds its nodes' entries)" if strong else
                                       f"hot values from a {synth.CONFIGS[3]['bindings']}-entry binding log per "
                                       "100k-node cell")
                                    + ", README default policy"),
                       "nodes_total": n_total, "nodes_per_gpu": N, "pods": P, "bindings_gpu0": B,
                       "parallelism": f"node-shard x{n_gpus}",
                       "engine": m["engine_path"] + (f" ({m['dispatch_note']})" if m.get("dispatch_note") else ""),
                       "batches_in_flight": m["K"],
                       "batch_times": (f"batch i at now0 + (i % {len(m['nows'])}) x {m['span'] / 1e9:g} s (its pods "
                                       "shifted alike): the hot-value cutoffs move every batch and K2's suffix "
                                       "search reruns; the cycle bounds the drift of the un-resynced synthetic "
                                       "snapshot and log")},
            "batches_in_flight": {"k": m["K"], "how": m["how"], "keys_agree": m["keys_agree"],
                                  "batch_latency_ms": round(m["batch_latency_ms"], 4)},
            "placements_per_s": round(placements, 1),
            "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
            "hot_value_refresh": {
                "form": "delta" if any(k.startswith("k2_delta") for k in kt) else "recount",
                "changed_bindings_mean": round(dl["mean"], 1), "changed_bindings_per_time": dl["per_time"],
                "anchor_now_ns": dl["anchor_now_ns"],
                "how": ("engine option k2_delta (time-ordered log): a slot's first refresh counts the widest window's "
                        "suffix (large form) as its anchor; each later batch reads only the bindings whose window rank "
                        "at its now differs from the anchor's and adjusts the anchor counts (kernel_ms, over the timed "
                        "batches' times in turn); re-anchors when they pass half the suffix or the log changes")},
            "allreduce_ms": None if m["ar_ms"] is None else round(m["ar_ms"], 4),
            "host": m["host"],
            "keys_match_1gpu": m["keys_match"],
            "keys_match_1gpu_how": m["keys_match_how"],
            "keys_match_stream": (all(b["stream"] for b in m["pinned"]) if m.get("pinned") else None),
            "keys_match_oracle_sample": (all(b["oracle_sample"] for b in m["pinned"]) if m.get("pinned") else None),
            "keys_pinned": m.get("pinned") and {
                "batches": m["pinned"],
                "how": ("the last timed batch and the one before it (another slot and `now`), as the timed path left "
                        "them: all keys == one engine over the whole cluster stepped on a HIP stream "
                        "(crane_dyn_step_keys_async, same pods and now); a 64-pod sample's chosen node (and score, "
                        "when the matrix fits) == the CPU oracle with the binding log's hot values at that now")},
            "roofline": roofline,
            "roofline_kernels": roofs,
            "roofline_cold": roofline_cold,
            "src_hash": shash,
            "lib_hash": lib_hash(),
            "cpu_baseline": cpu,
            "greedy": greedy,
            "host_parse": host_parse,
            "chosen_sample": [int(x) for x in keys[:4]],
        }
        line.update(extras)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
