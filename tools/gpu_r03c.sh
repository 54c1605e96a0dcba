# large-form K2 A/B on the cold leg (k2x_threads), parity of the hot-value tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "hot_values" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for t in 512 256 1024; do
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 --opt k2x_threads=$t > $O/cold_$t.log 2>&1 || { tail -30 $O/cold_$t.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold_$t.log').read().strip().splitlines()[-1]); print($t, d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'], d['k1']['ms'], d['k1']['frac'])"
done
