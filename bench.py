"""Benchmark of the Dynamic-plugin hot path on MI355X (BASELINE.json config 3 per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one scheduling batch of the reference's hot path over one shard:
  K2 hot values from the shard's 1M-entry binding log (binding.go:81-97, node.go:113-121)
  K1 node pass over the shard's parsed annotations (stats.go:51-112 pod-invariant parts)
  K3 Filter + Score + argmax for every (pod, node) pair (plugins.go:39-98, selectHost)
  RCCL int64 max all-reduce of the per-pod packed keys across node shards (N > 1)
Each rank owns config 3's 100k nodes (node indices rank*100k + i) and every
rank scores the same 10k pods: weak scaling, value = pods * total nodes / step.
Inputs are resident in HBM before timing; data is synthetic (crane_dyn/synth.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "crane-scheduler_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_pmc_summary.json")
# engine stage name -> kernel name in the rocprofv3 PMC summary (templates: prefix + suffix)
STAGE_KERNEL = {
    "k1_node_pass+k3a_steps": ("crane::k1_node_pass<", "true>"),
    "k1_node_pass": ("crane::k1_node_pass<", "false>"),
    "k2x_partition": ("crane::k2x_partition", None),
    "k2x_partition+k3p_pods": ("crane::k2x_pods", None),
    "k2x_dedupe+k3p_pods": ("crane::k2x_dedupe_pods", None),
    "k2x_dedupe": ("crane::k2x_dedupe", None),
    "k2y_bin_hist": ("crane::k2y_bin_hist", None),
    "k3p_pods": ("crane::k3p_pods", None),
}


def _stage_match(name, kernel):
    pre, suf = STAGE_KERNEL.get(name, (None, None))
    if pre is None:
        return False
    return kernel == pre if suf is None else kernel.startswith(pre) and kernel.endswith(suf)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--cpu-pods", type=int, default=1920, help="pods in the bounded CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16, help="upstream kube-scheduler parallelism")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-greedy", action="store_true", help="skip the config-5 sequential-greedy measurement")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as a captured graph (measured slower than eager launches on ROCm 7.2)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import crane_dyn as cd
    from crane_dyn import synth

    cfg = synth.CONFIGS[args.config]
    N, P, B = cfg["nodes"], cfg["pods"], cfg["bindings"]
    if args.config == 4:  # 1M nodes x 100k pods over 8 GPUs: one rank holds N/8
        N = N // 8
    spec = cd.default_policy_spec()
    c = synth.make_cluster(spec, N, P, n_bindings=B, seed=20250215 + args.config * 1000 + rank)
    # the pod batch is the same on every shard (only nodes and bindings are per rank)
    c.now, c.ds = synth.make_pods(P, seed=20250215 + args.config)
    eng = cd.Engine(cd.Policy(spec), local)
    val, ts, _ = c.rows(eng.metric_names)
    eng.upload_nodes(val, ts, c.hv, c.hv_ts, node_offset=rank * N)
    eng.upload_bindings(c.b_node, c.b_ts)
    d_now = torch.from_numpy(c.now).to(dev)
    d_flags = torch.from_numpy(c.ds).to(dev)
    d_keys = torch.empty(P, dtype=torch.int64, device=dev)
    now_sync = int(synth.NOW0_NS)

    # a dedicated stream: the default stream's handle is 0, which the C ABI reads as "engine stream"
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(e=None, collective=True):
        if e:
            e[0].record(stream)
        # K2 (k2x, k2y) + K3p on a second queue, then K1+K3a (fused node pass), K3s
        eng.step_keys_async(now_sync, now_sync, d_now, d_flags, d_keys, sh)
        if e:
            e[1].record(stream)
        if world > 1 and collective:
            dist.all_reduce(d_keys, op=dist.ReduceOp.MAX)       # RCCL over xGMI
        if e:
            e[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # per-stage times from eager passes: HIP events around the engine call, and the
    # engine's own per-kernel events (crane_dyn_set_profiling; while it is on, the
    # engine runs the step's kernels back to back on one queue)
    eng.set_profiling(True)
    stages = {}
    for k in range(args.steps):
        step(ev[k])
        for name, t in eng.stage_times():
            stages.setdefault(name, []).append(t)
    eng.set_profiling(False)
    torch.cuda.synchronize(dev)
    graph = None
    if args.graph:
        # one scheduling batch = one graph replay: K2 + K1 + K3 launches captured once,
        # inputs (pods, binding log, node SoA) stay in device buffers updated in place
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            step(collective=False)
        graph.replay()
        torch.cuda.synchronize(dev)

    def timed_step():
        if graph is None:
            step()
        else:
            graph.replay()
            if world > 1:
                dist.all_reduce(d_keys, op=dist.ReduceOp.MAX)  # RCCL over xGMI

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        timed_step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed * 1e3 / args.steps
    step_ms_prof = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    ar_ms = float(np.mean([b.elapsed_time(c_) for _, b, c_ in ev]))
    stage_ms = {k: float(np.mean(v)) for k, v in stages.items()}

    keys = d_keys.cpu().numpy()
    evals = P * N * world
    value = evals / (ms_step / 1e3)
    placements = P / (ms_step / 1e3)

    # Rooflines per kernel stage: ALGORITHMIC bytes per launch / the
    # stage's mean duration from the engine's HIP events above.  The dominant stage is `roofline`.
    M = len(eng.metric_names)
    W = len(spec["hotValue"])
    PD, PR = len(spec["predicate"]), len(spec["priority"])
    pd_, pr_ = (4, 6) if PD <= 4 and PR <= 6 else ((8, 8) if PD <= 8 and PR <= 8 else (16, 16))
    rec_bytes = -(-(24 + 16 * pr_ + 8 + 8 * pd_) // 16) * 16  # sizeof(NodeRec<PD,PR>)
    max_tr_s = max(tr for tr, _ in spec["hotValue"]) // 10**9
    b_in = int((c.b_ts > now_sync // 10**9 - max_tr_s).sum())  # bindings inside the widest window
    # the fused keys-only node pass leaves the records in LDS (CRANE_K1_KEEP_REC=1 writes them)
    keep_rec = os.environ.get("CRANE_K1_KEEP_REC") == "1"
    k2x_b = B * 12 + b_in * 4
    k3p_b = P * (8 + 1 + 4 + 8 + 8)
    # dedupe-form K2: one 4-byte entry per distinct (2048-binding region, node, window rank),
    # a (count, offset) pair per (node block, region); the node pass reads both
    dedupe = os.environ.get("CRANE_K2", "dedupe") == "dedupe"
    cut = np.sort(np.array([now_sync // 10**9 - tr // 10**9 for tr, _ in spec["hotValue"]], np.int64))
    jr = (c.b_ts[:, None] > cut[None, :]).sum(1)
    okb = (jr > 0) & (c.b_node >= 0) & (c.b_node < N)
    reg = np.arange(B, dtype=np.int64) // 2048
    E = int(np.unique((reg[okb] * (N + 1) + c.b_node[okb]) * 8 + jr[okb] - 1).size) if B else 0
    k1_bs = int(os.environ.get("CRANE_K1_THREADS", "256"))
    co_b = 8 * (-(-N // k1_bs)) * (-(-B // 2048))
    k2d_b = B * 12 + E * 4 + co_b
    alg = {
        "k2x_dedupe": (k2d_b, "bindings read + distinct (region, node, bucket) entries + count/offset written"),
        "k2x_dedupe+k3p_pods": (k2d_b + k3p_b, "bindings read + distinct entries + count/offset written; pod now + "
                                               "flag read, partition + keys written"),
        "k2x_partition": (k2x_b, "bindings read (int32 node + int64 ts) + kept entries written"),
        "k2x_partition+k3p_pods": (k2x_b + k3p_b, "bindings read + kept entries written; pod now + flag read, "
                                                  "partition + keys written"),
        "k2y_bin_hist": (b_in * 4 + 4 * W * N, "kept entries read + window counts added"),
        "k1_node_pass+k3a_steps": ((N * (16 * M + 8 + (rec_bytes if keep_rec else 0))
                                    + (E * 4 + co_b if dedupe else N * 8 * W)),
                                   "SoA (value, ts) read + hot value written + "
                                   + ("K2 entries and count/offset read" if dedupe else "buckets read and zeroed")
                                   + (" + NodeRec written" if keep_rec else "")),
        "k1_node_pass": (N * (16 * M + 8 * W + rec_bytes + 8), "SoA + buckets + NodeRec + hot value"),
        "k3p_pods": (k3p_b, "pod now + flag read, partition + keys written"),
    }
    roofs = {}
    for name, t in stage_ms.items():
        if name in alg and t > 0:
            gbs = alg[name][0] / (t * 1e-3) / 1e9
            roofs[name] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(gbs / HBM_PEAK_GBS, 4), "ms": round(t, 4),
                           "alg_bytes": int(alg[name][0]), "bytes": alg[name][1]}
    dom = max(stage_ms, key=stage_ms.get) if stage_ms else None
    # HBM traffic per launch from the committed PMC summary of this bench
    # (tools/gpu_pmc.sh: separate FETCH_SIZE / WRITE_SIZE passes, KiB, FETCH_SIZE x2 on gfx950)
    pmc = {}
    if os.path.exists(PMC_SUMMARY):
        pmc = json.load(open(PMC_SUMMARY))
    for name, e in roofs.items():
        hits = [v for k, v in pmc.items() if _stage_match(name, k) and "traffic_bytes" in v]
        e["traffic"] = int(hits[0]["traffic_bytes"]) if hits else None
    roof = None
    if dom in roofs:
        roof = dict(roofs[dom], kernel=dom)
        if roof.get("traffic") is not None:
            roof["traffic_source"] = os.path.relpath(PMC_SUMMARY, ROOT)
    elif dom:
        roof = {"bound": None, "kernel": dom, "ms": round(stage_ms[dom], 4), "note": "no HBM roofline for this stage"}
    greedy = None
    if world == 1 and not args.no_greedy:
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
    host_parse = ctl = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        cp = min(args.cpu_pods, P)
        ann = c.annotations()
        t1 = time.perf_counter()
        _, _, och = O.eval_strings(spec, ann, c.now[:cp], c.ds[:cp], threads=args.cpu_threads, want_matrix=False)
        dt = time.perf_counter() - t1
        cpu = {"value": round(cp * N / dt, 1), "unit": "pod-node evals/s", "cores": args.cpu_threads, "kind": "port",
               "sample": f"{cp} pods x {N} nodes, string mode (re-parse every annotation per call like stats.go), "
                         f"{args.cpu_threads} threads, {dt:.1f}s"}
        # the stronger CPU data point, pre-parsed SoA (no string work per call)
        okr = c.rows(eng.metric_names)[2]
        t1 = time.perf_counter()
        O.eval_soa(spec, eng.metric_names, okr, val, ts, np.ones(N, np.uint8), c.hv, c.hv_ts, c.now[:cp], c.ds[:cp],
                   threads=args.cpu_threads, want_matrix=False)
        dts = time.perf_counter() - t1
        cpu["soa_mode"] = {"value": round(cp * N / dts, 1), "unit": "pod-node evals/s", "cores": args.cpu_threads,
                           "sample": f"{cp} pods x {N} nodes, pre-parsed SoA, {dts:.1f}s"}
        # the once-per-sync host parse of the same snapshot's annotation
        # strings into the SoA the engine uploads (crane_parse_annotations, C++ threads)
        snap = cd.SnapshotStrings(eng.metric_names, ann)
        host_parse = {"strings": len(snap), "nodes": N}
        for label, th in (("threads_16", args.cpu_threads), ("threads_all", 0)):
            snap.parse(synth.SHANGHAI, th)
            reps = []
            for _ in range(3):
                t1 = time.perf_counter()
                snap.parse(synth.SHANGHAI, th)
                reps.append(time.perf_counter() - t1)
            dtp = float(np.median(reps))
            host_parse[label] = {"ms_per_sync": round(dtp * 1e3, 2), "strings_per_s": round(len(snap) / dtp, 1)}
        # the controller's per-sync hot-value annotation pass
        # (node.go:113-121 over binding.go:81-97) as K2+K1 plus the 8 B/node readback,
        # checked bit-exact against the oracle's count over the full binding log
        eng.refresh_hot_values(now_sync)
        eng.hot_values()
        reps = []
        for _ in range(5):
            t1 = time.perf_counter()
            eng.refresh_hot_values(now_sync)
            ghv = eng.hot_values()
            reps.append(time.perf_counter() - t1)
        t1 = time.perf_counter()
        _, ohv = O.hot_values(spec, c.b_node, c.b_ts, N, now_sync // 10**9)
        ocpu = time.perf_counter() - t1
        ctl = {"workload": f"{B}-entry binding log -> {N} node hot values", "gpu_ms": round(float(np.median(reps)) * 1e3, 3),
               "timing": "host wall incl. K2 + K1 + D2H of hot values", "oracle_cpu_ms": round(ocpu * 1e3, 2),
               "oracle": "C restatement, one pass over the log (the reference scans the log once per node: O(N*B))",
               "matches_oracle": bool(np.array_equal(ghv, ohv.astype(np.float64)))}
        pv, pt, _, _ = snap.soa()
        okm = c.rows(eng.metric_names)[2].astype(bool)
        host_parse["matches_generator_soa"] = bool(np.array_equal(pt[okm], ts[okm]) and np.array_equal(pv[okm],
                                                                                                       val[okm]))
    if rank == 0:
        line = {
            "metric": "pod-node filter+score evals/sec",
            "value": round(value, 1),
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"config{args.config}: {N} nodes/GPU x {P} pods, 6 metrics, hot values from "
                                   f"{B}-entry binding log per GPU, README default policy",
                       "nodes_per_gpu": N, "pods": P, "bindings_per_gpu": B, "parallelism": f"node-shard x{world}",
                       "launch": "eager" if graph is None else "hipGraph replay per batch"},
            "placements_per_s": round(placements, 1),
            "kernel_ms": {"step_profiled_serial": round(step_ms_prof, 4), "allreduce": round(ar_ms, 4)},
            "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
            "roofline": roof,
            "roofline_stages": roofs,
            "cpu_baseline": cpu,
            "greedy": greedy,
            "host_parse": host_parse,
            "controller_hot_values": ctl,
            "chosen_sample": [int(x) for x in keys[:4]],
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
