# K1 probe: step/select parity tests, cold 4M-node stream bench, step traces configs 3/4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_select.py tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
timeout -k 10 300 python tools/stream_bench.py --k2 auto > $OUT/stream.json 2> $OUT/stream.err || { tail -20 $OUT/stream.err; exit 1; }
timeout -k 10 120 python tools/trace_step.py --config 3 > $OUT/trace3.json || exit 1
timeout -k 10 120 python tools/trace_step.py --config 4 > $OUT/trace4.json || exit 1
tail -1 $OUT/pytest.log
