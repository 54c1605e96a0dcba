# Split node pass check: step parity tests, full GPU suite, cold 4M stream (auto / fused), bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_step.log 2>&1 || { tail -40 $O/pytest_step.log; exit 1; }
tail -1 $O/pytest_step.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/stream_bench.py --k2 auto > $O/stream.json 2> $O/stream.err || { tail $O/stream.err; exit 1; }
timeout -k 10 200 python tools/stream_bench.py --k2 auto --opt k1_split=0 > $O/stream_fused.json 2> $O/stream_fused.err || { tail $O/stream_fused.err; exit 1; }
cat $O/stream.json $O/stream_fused.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-greedy --no-extras > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --no-greedy --no-extras > $O/bench4.log 2>&1 || { tail $O/bench4.log; exit 1; }
tail -1 $O/bench.log | cut -c1-700
tail -1 $O/bench4.log | cut -c1-1400
