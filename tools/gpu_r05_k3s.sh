# Same-box A/B of K3s builds at config 3: crane-scheduler_amd/lib_ab/lib_<V>.so swapped in as the
# engine library; step tests on the first variant's first round, then per variant and round the
# in-flight probe (1 and 4 batches) and the config-3 phase trace.
#   bash tools/gpu_r05_k3s.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
if [ -n "$AB_TESTS" ]; then
  cp crane-scheduler_amd/lib_ab/lib_$AB_TESTS_LIB.so $L || exit 1
  timeout -k 10 400 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
  echo "$AB_TESTS_LIB: $(tail -1 $O/pytest.log)"
fi
for rep in 1 2; do
  for v in "$@"; do
    cp crane-scheduler_amd/lib_ab/lib_$v.so $L || exit 1
    timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --steps 400 > $O/inf_${v}_$rep.json 2>&1 || { tail $O/inf_${v}_$rep.json; exit 1; }
    timeout -k 10 200 python tools/trace_step.py --config 3 --reps 7 > $O/t3_${v}_$rep.json 2> $O/t3_${v}_$rep.err || { tail $O/t3_${v}_$rep.err; exit 1; }
    python3 - "$O" "$v" "$rep" <<'PY'
import json, sys
o, v, r = sys.argv[1:4]
inf = json.loads(open(f"{o}/inf_{v}_{r}.json").read().strip().splitlines()[-1])
t = json.load(open(f"{o}/t3_{v}_{r}.json"))
k = t["K3s"]
print(v, r, "c3 ms/batch 1/4 in flight:", inf["inflight1"]["ms_per_step"], inf["inflight4"]["ms_per_step"],
      "| K3s span", k["span"], "end p90", k["end"]["p90"], "phases", {p: q["med"] for p, q in k["phases"].items()},
      "| K1 span", t["K1"]["span"])
PY
  done
done
