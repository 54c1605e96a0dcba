# large-form K2 A/B: partition workgroup width and count/offset layout (cold leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "hot_values" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for o in "k2l_threads=512 k2l_co_t=0" "k2l_threads=512 k2l_co_t=1" "k2l_threads=1024 k2l_co_t=1"; do
  set -- $o
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 --opt $1 --opt $2 > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold.log').read().strip().splitlines()[-1]); print('$o', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'], d['k1']['ms'], d['k1']['frac'])"
done
timeout -k 10 300 python tools/trace_k2l.py --opt k2l_co_t=1 2>/dev/null | tail -1
