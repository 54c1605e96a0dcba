# Round-4 end-of-round evidence on the current tree, in two stages (one gpurun call each):
#   bash tools/gpu_final_r04.sh <tag> verify   GPU suite, smoke, default bench line, rocprof kernel
#                                              stats of the bench (4 in flight) and of one batch alone
#   bash tools/gpu_final_r04.sh <tag> lines    PMC passes for config 3 and the cold leg on these kernel
#                                              sources, installed under profiles/pmc/ on the box, then
#                                              the bench lines carrying their traffic (default, config 4),
#                                              the collective rehearsed on one rank, --gpus 2 refusal
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r04f}
O=gpurun_out/$T
mkdir -p $O
H=$(python3 -c "import bench; print(bench.src_hash())")
echo "src_hash $H"
export TMPDIR=/tmp
case $2 in
verify)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-600
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o bench \
      -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-greedy > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof1 -o bench1 \
      -- python3 $GRAFT_REPO_ROOT/bench.py --inflight 1 --no-cpu-baseline --no-greedy --no-extras > $O/prof1.log 2>&1 || { tail -20 $O/prof1.log; exit 1; }
  python3 tools/kstats.py $O/prof/bench_kernel_stats.csv
  python3 tools/kstats.py $O/prof1/bench1_kernel_stats.csv
  ;;
lines)
  bash tools/gpu_pmc.sh $T "3 cold" || { echo "pmc failed"; exit 1; }
  mkdir -p $O/pmc_json profiles/pmc
  for c in 3 cold; do cp gpurun_out/pmc_${T}_$c/summary.json $O/pmc_json/config${c}_$H.json && cp $O/pmc_json/config${c}_$H.json profiles/pmc/; done
  timeout -k 10 600 python bench.py > $O/bench_traffic.log 2>&1 || { tail $O/bench_traffic.log; exit 1; }
  timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > $O/bench4.log 2>&1 || { tail $O/bench4.log; exit 1; }
  WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 300 python -u bench.py --config 3 \
      --rehearse-collective --no-extras --no-cpu-baseline --no-greedy --steps 512 > $O/rehearse3.log 2>&1 || { tail -30 $O/rehearse3.log; exit 1; }
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 512 > $O/nocoll3.log 2>&1 || { tail -30 $O/nocoll3.log; exit 1; }
  timeout -k 10 120 python bench.py --gpus 2 --no-extras > $O/gpus2.log 2>&1
  echo "gpus2 exit $?: $(tail -1 $O/gpus2.log)"
  python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_traffic", "bench4", "rehearse3", "nocoll3"):
    d = json.loads(open(f"{o}/{f}.log").read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    rc = d.get("roofline_cold") or {}
    print(f, d["value"], d["ms_per_step"], "roof", r.get("frac"), r.get("traffic"),
          "cold", {k: (v["frac"], v["traffic"]) for k, v in rc.items() if isinstance(v, dict) and "frac" in v},
          "ar", d.get("allreduce_ms"), d.get("keys_match_1gpu"), "host", d.get("host"))
PY
  ;;
*) echo "stage: verify | lines"; exit 2;;
esac
echo "src_hash $H"
