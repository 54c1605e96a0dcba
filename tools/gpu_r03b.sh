# large-form K2: hot-value parity (all forms) + the cold-leg roofline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "hot_values" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --leg cold --steps 5 > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
tail -1 $O/cold.log
