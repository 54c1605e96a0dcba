"""Print DESIGN.md §9's table rows from a round's kept bench lines (profiles/<tag>_bench*.json,
the drop-in probe, the cold-leg sweep) so the doc quotes exactly what is kept.

    python tools/design_table.py <tag>      e.g. r03_fin
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]


def line(name):
    p = os.path.join(ROOT, "profiles", f"{tag}_{name}.json")
    return json.loads(open(p).read().strip().splitlines()[-1]) if os.path.exists(p) else None


b3, b4, r3 = line("bench"), line("bench_config4"), line("rehearse3")
rows = []
k = b3["kernel_ms"]
rows.append(("config 3 step (100k nodes × 10k pods, hot values from a 1M-entry log), 4 batches in flight",
             f"**{b3['ms_per_step']} ms/batch → {b3['value']:.2e} pod-node pairs resolved/s (full-rescan equivalent), "
             f"{b3['placements_per_s']:.2e} placements/s**"))
rows.append(("one batch alone (latency) and its kernels",
             f"{b3['batches_in_flight']['batch_latency_ms']} ms: " + ", ".join(f"{n} {v * 1e3:.1f} µs" for n, v in k.items())))
r = b3["roofline"]
rows.append(("K1 vs HBM, config 3 (the line's `roofline`)",
             f"{r['alg_bytes'] / 1e6:.1f} MB / {r['ms'] * 1e3:.1f} µs = {r['achieved']:.0f} GB/s = {r['frac']:.3f} of 8 TB/s; "
             f"PMC traffic {r['traffic'] / 1e6 if r['traffic'] else float('nan'):.1f} MB"))
c = b3["roofline_cold"]
for key, what in (("k2", "K2 (large form) cold, 4M nodes × 16M bindings"), ("k1", "K1 fused with the step tables, cold 4M"),
                  ("k1_records", "K1 writing records (matrix / greedy / selection / drop-in paths), cold 4M")):
    if key not in c:
        continue
    x = c[key]
    tr = f"; PMC traffic {x['traffic'] / 1e6:.0f} MB" if x.get("traffic") else ""
    rows.append((what, f"{x['ms']} ms, {x['alg_bytes'] / 1e6:.0f} MB algorithmic → {x['achieved'] / 1e3:.2f} TB/s = "
                       f"**{x['frac']:.2f}** of 8 TB/s{tr}"))
if b4:
    rows.append(("config 4 on one GPU (1M nodes × 100k pods), 4 in flight",
                 f"{b4['ms_per_step']} ms/batch ({b4['batches_in_flight']['batch_latency_ms']} alone: " +
                 ", ".join(f"{n} {v * 1e3:.0f} µs" for n, v in b4["kernel_ms"].items()) + f") → {b4['value']:.2e} pairs/s"))
if r3:
    rows.append(("collective path rehearsed on one rank (config 3, all-reduce per 64 batches)",
                 f"{r3['ms_per_step']} ms/batch; all-reduce {r3['allreduce_ms']} ms per call; keys_match_1gpu "
                 f"{r3['keys_match_1gpu']}"))
for key, what in (("matrix_config2", "config 2 full matrices (5000 × 1000, K3m)"),
                  ("matrix_config3", "config 3 full matrices (2 × 1 GB int8)")):
    x = b3[key]
    rows.append((what, f"{x['kernel_ms']['k3m_matrix+keys'] * 1e3:.1f} µs kernel, {x['evals_per_s']:.2e} pairs/s with "
                       f"every pair in HBM; {x['roofline']['frac']:.2f} of 8 TB/s"))
d = b3["dropin"]
bd = d["breakdown"]
rows.append(("drop-in cycle at 100k nodes (Filter on every node + Score on the feasible ones, 16 threads, + selectHost)",
             f"{d['dropin_ms_per_pod']} ms per pod (Filter fan-out {bd['filter_fanout_ms']}, Score fan-out "
             f"{bd['score_fanout_ms']}, selectHost {bd['select_ms']} ms; the pool's own no-op fan-outs "
             f"{bd['harness_noop_fanouts_ms']} ms); CPU plugin in the same harness {d.get('cpu_same_harness_ms_per_pod')} ms "
             f"({d.get('speedup_vs_cpu_same_harness')}×); chosen nodes equal the engine's: {d['matches_engine_chosen']}"))
x = b3["controller_hot_values"]
rows.append(("controller hot values (1M-entry heap → 100k nodes)",
             f"append + GC + refresh + readback {x['append_sync_ms']} ms; full re-upload {x['full_replace_sync_ms']} ms; "
             f"CPU oracle {x['oracle_cpu_ms']} ms; bit-exact: {x['matches_oracle']}"))
x = b3["host_parse"]
rows.append(("host parse of a config-3 snapshot (700k strings)", f"{x['threads_16']['ms_per_sync']} ms per sync (16 threads)"))
x = b3["greedy"]
rows.append(("config 5 greedy (100k × 50k)", f"{x['ms']} ms → {x['placements_per_s']:.2e} placements/s"))
x = b3["select_config3"]
rows.append(("selection, config-3 queue (shipped profile)",
             f"adaptive 5 % windows {x['adaptive_percentage']['ms']} ms per 10k-pod queue (walk "
             f"{x['adaptive_percentage']['kernel_ms'].get('k_sel_chain_rs')} ms); every node scored "
             f"{x['percentage_100']['ms']} ms"))
x = b3["cpu_baseline"]
rows.append((f"CPU baseline (oracle string mode, {x['cores']} threads, {x['cpu_model']})",
             f"{x['value']:.2e} evals/s; pre-parsed SoA mode {x['soa_mode']['value']:.2e}"))
print("| what | value |\n|---|---|")
for a, b in rows:
    print(f"| {a} | {b} |")
