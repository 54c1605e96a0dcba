# Round-end evidence on the current tree, in stages (each fits one gpurun call):
#   bash tools/gpu_final.sh <tag> verify   GPU suite + smoke + bench + cold stream + rocprof stats (gpu_verify.sh)
#   bash tools/gpu_final.sh <tag> pmc "3 cold 4"   PMC summaries of those workloads for these kernel sources
#                                                  (gpurun_out/<tag>/pmc_json/config<C>_<hash>.json: commit them
#                                                  under profiles/pmc/ so bench lines on these sources carry traffic)
#   bash tools/gpu_final.sh <tag> lines    bench lines with the traffic attached (config 3 with every leg,
#                                          config 4), the collective rehearsed on one rank, `--gpus 2` on
#                                          this one-GPU box (must refuse, not report one rank)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
H=$(python3 -c "import bench; print(bench.src_hash())")
mkdir -p gpurun_out/$T
case $2 in
verify)
    bash tools/gpu_verify.sh $T || exit 1;;
pmc)
    bash tools/gpu_pmc.sh $T "$3" || exit 1
    mkdir -p gpurun_out/$T/pmc_json
    for c in $3; do cp gpurun_out/pmc_${T}_$c/summary.json gpurun_out/$T/pmc_json/config${c}_$H.json; done;;
lines)
    timeout -k 10 600 python bench.py > gpurun_out/$T/bench_traffic.log 2>&1 || { tail gpurun_out/$T/bench_traffic.log; exit 1; }
    timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/$T/bench4_traffic.log 2>&1 \
        || { tail gpurun_out/$T/bench4_traffic.log; exit 1; }
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
    ;;
*) echo "stage: verify | pmc <workloads> | lines"; exit 2;;
esac
echo "hash $H"
