# K1 change check: step / engine / shard / select parity tests, cold 4M stream (read flush),
# K1 phase traces at config 3 and 4M, bench (one batch + in flight).  Usage: bash tools/gpu_k1_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/stream_bench.py --k2 auto > $O/stream.json 2> $O/stream.err || { tail $O/stream.err; exit 1; }
cat $O/stream.json
timeout -k 10 200 python tools/trace_step.py --config 3 > $O/trace3.json 2> $O/trace3.err || { tail $O/trace3.err; exit 1; }
timeout -k 10 200 python tools/trace_step.py --config 3 --nodes 4000000 --bindings 16000000 > $O/trace4m.json 2> $O/trace4m.err || { tail $O/trace4m.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-greedy --no-extras > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1500
