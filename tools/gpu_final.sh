# Round-end evidence on the current tree: GPU suite + smoke + bench + stream + rocprof stats
# (tools/gpu_verify.sh), PMC summaries of configs 3, cold, 4, 2, 3m, 4m for these kernel
# sources (tools/gpu_pmc.sh), then the config-3 and config-4 bench lines with that traffic
# attached, the collective path rehearsed on one rank, and `--gpus 2` on this one-GPU box
# (must refuse, not report one rank).
#   bash tools/gpu_final.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
H=$(python3 -c "import bench; print(bench.src_hash())")
bash tools/gpu_verify.sh $T || exit 1
bash tools/gpu_pmc.sh $T "3 cold 4 2 3m 4m" || exit 1
for c in 3 cold 4 2 3m 4m; do cp gpurun_out/pmc_${T}_$c/summary.json profiles/pmc/config${c}_$H.json; done
mkdir -p gpurun_out/$T/pmc_json && cp profiles/pmc/config*_$H.json gpurun_out/$T/pmc_json/
timeout -k 10 600 python bench.py > gpurun_out/$T/bench_traffic.log 2>&1 || { tail gpurun_out/$T/bench_traffic.log; exit 1; }
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/$T/bench4_traffic.log 2>&1 || { tail gpurun_out/$T/bench4_traffic.log; exit 1; }
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 300 python -u bench.py --config 3 \
    --rehearse-collective --no-extras --no-cpu-baseline --no-greedy > gpurun_out/$T/rehearse3.log 2>&1 \
    || { tail -30 gpurun_out/$T/rehearse3.log; exit 1; }
timeout -k 10 120 python bench.py --gpus 2 --no-extras > gpurun_out/$T/gpus2.log 2>&1
echo "gpus2 exit $?: $(tail -1 gpurun_out/$T/gpus2.log)"
python3 - "$T" <<'PY'
import json, sys
t = sys.argv[1]
for f in ("bench_traffic", "bench4_traffic", "rehearse3"):
    d = json.loads(open(f"gpurun_out/{t}/{f}.log").read().strip().splitlines()[-1])
    r = d["roofline"] or {}
    rc = d.get("roofline_cold") or {}
    print(f, d["ms_per_step"], d["kernel_ms"], "roof", r.get("frac"), r.get("traffic"),
          "cold", {k: (v["frac"], v["traffic"]) for k, v in rc.items() if isinstance(v, dict) and "frac" in v},
          "ar", d.get("allreduce_ms"), d.get("keys_match_1gpu"))
PY
echo "hash $H"
