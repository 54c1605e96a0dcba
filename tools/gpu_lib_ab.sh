# Same-box A/B of engine builds: crane-scheduler_amd/lib_ab/lib_<V>.so swapped in as the
# engine library, per variant the config-3 in-flight probe, config-4 (one GPU) bench kernel
# times and the config-4-shard trace spans.   Usage: bash tools/gpu_lib_ab.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
# the product library comes back however the script ends (timeouts, signals, errors)
trap 'cp $O/orig.so $L' EXIT
for v in "$@"; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L || { cp $O/orig.so $L; exit 1; }
  if [ -n "$AB_TESTS" ]; then  # parity of the variant first (e.g. AB_TESTS=tests/test_step_gpu.py)
    timeout -k 10 300 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 \
      || { tail -20 $O/pytest_$v.log; cp $O/orig.so $L; exit 1; }
    echo "$v: $(tail -1 $O/pytest_$v.log)"
  fi
  timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 > $O/inf_$v.json 2>&1 || { tail $O/inf_$v.json; cp $O/orig.so $L; exit 1; }
  timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --no-greedy --no-extras > $O/b4_$v.log 2>&1 || { tail $O/b4_$v.log; cp $O/orig.so $L; exit 1; }
  timeout -k 10 200 python tools/trace_step.py --config 4 > $O/t4_$v.json 2> $O/t4_$v.err || { tail $O/t4_$v.err; cp $O/orig.so $L; exit 1; }
  python3 - "$O" "$v" <<'PY'
import json, sys
o, v = sys.argv[1], sys.argv[2]
inf = json.loads(open(f"{o}/inf_{v}.json").read().strip().splitlines()[-1])
b4 = json.loads(open(f"{o}/b4_{v}.log").read().strip().splitlines()[-1])
t4 = json.load(open(f"{o}/t4_{v}.json"))
print(v, "c3 1/4:", inf["inflight1"]["ms_per_step"], inf["inflight4"]["ms_per_step"], "| c4:", b4["ms_per_step"],
      b4["batches_in_flight"]["batch_latency_ms"], b4["kernel_ms"].get("k3s_eval"), "| c4 shard K3s span:", t4["K3s"]["span"])
PY
done
cp $O/orig.so $L
