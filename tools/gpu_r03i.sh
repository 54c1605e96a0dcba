# selection chain (LDS rank/select) parity + timing; large-K2 Y gather A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_select.py tests/test_engine_gpu.py -k "select or hot_values" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in sel_chain=0 sel_chain=1; do
  timeout -k 10 300 python tools/select_probe.py $v > $O/sel_$v.json 2>&1 || { tail $O/sel_$v.json; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/sel_$v.json').read().strip().splitlines()[-1]); print('$v', d['adaptive_percentage']['ms'], d['adaptive_percentage']['kernel_ms'], d['percentage_100']['ms'])"
done
for o in "k2l_co_t=0" "k2l_co_t=1"; do
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 --opt $o > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold.log').read().strip().splitlines()[-1]); print('$o', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'], d['k1']['ms'], d['k1']['frac'])"
done
timeout -k 10 300 python tools/trace_k2l.py --opt k2l_co_t=1 2>/dev/null | tail -1
