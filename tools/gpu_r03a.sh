set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_bindings.py tests/test_greedy_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --rehearse-collective --steps 40 --no-extras --no-cpu-baseline --no-greedy > $O/rehearse.log 2>&1 || { tail -30 $O/rehearse.log; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --config 4 --rehearse-collective --steps 20 --no-extras --no-cpu-baseline --no-greedy > $O/rehearse4.log 2>&1 || { tail -30 $O/rehearse4.log; exit 1; }
python - <<'PY'
import json
for f in ("bench","rehearse","rehearse4"):
    d=json.loads(open(f"gpurun_out/r03a/{f}.log").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("keys_match_1gpu"), json.dumps(d.get("roofline_cold"))[:900])
PY
