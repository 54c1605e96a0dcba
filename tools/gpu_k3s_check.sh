# K3s check: step parity tests, config-3 and config-4-shard traces, config-3 / config-4 bench (no extras).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/trace_step.py --config 3 > $O/trace3.json 2> $O/trace3.err || { tail $O/trace3.err; exit 1; }
timeout -k 10 200 python tools/trace_step.py --config 4 > $O/trace4.json 2> $O/trace4.err || { tail $O/trace4.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-greedy --no-extras > $O/bench3.log 2>&1 || { tail $O/bench3.log; exit 1; }
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --no-greedy --no-extras > $O/bench4.log 2>&1 || { tail $O/bench4.log; exit 1; }
python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("trace3", "trace4"):
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d.get("nodes"), {k: d[k]["span"] for k in d if isinstance(d[k], dict) and "span" in d[k]})
for f in ("bench3", "bench4"):
    d = json.loads(open(f"{o}/{f}.log").read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["batches_in_flight"]["batch_latency_ms"], d["kernel_ms"])
PY
