# Same-box A/B of engine builds on the headline and the cold legs: crane-scheduler_amd/lib_ab/lib_<V>.so
# swapped in; per variant the step/engine parity tests, the config-3 in-flight probe (1 and 4
# batches) and the cold 4M-node K1/K2 leg.   Usage: bash tools/gpu_lib_ab2.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for rep in 1 2; do
for v in "$@"; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L || exit 1
  if [ $rep = 1 ]; then
    timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 \
      || { tail -20 $O/pytest_$v.log; exit 1; }
    echo "$v: $(tail -1 $O/pytest_$v.log)"
  fi
  timeout -k 10 200 python tools/inflight_probe.py --bound --inflight 1,4 > $O/inf_${v}_$rep.json 2>&1 || { tail $O/inf_${v}_$rep.json; exit 1; }
  timeout -k 10 300 python bench.py --leg cold --steps 7 > $O/cold_${v}_$rep.json 2> $O/cold_${v}_$rep.err || { tail $O/cold_${v}_$rep.err; exit 1; }
  python3 - "$O" "$v" "$rep" <<'PY'
import json, sys
o, v, r = sys.argv[1], sys.argv[2], sys.argv[3]
inf = json.loads(open(f"{o}/inf_{v}_{r}.json").read().strip().splitlines()[-1])
c = json.load(open(f"{o}/cold_{v}_{r}.json"))
print(v, r, "c3 1/4:", inf["inflight1"]["ms_per_step"], inf["inflight4"]["ms_per_step"], "host", inf["inflight4"]["host_enqueue_ms_per_step"],
      "| cold k1", c["k1"]["ms"], c["k1"]["frac"], "k2", c["k2"]["ms"], "k2ts", c["k2_timestamp_path"]["ms"], "k1r", c["k1_records"]["ms"])
PY
done
done
