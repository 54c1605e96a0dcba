# selection chain + node tables + plugin: parity; selection timing; drop-in leg; Y gather A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_select.py tests/test_engine_gpu.py tests/test_plugin_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in sel_chain=0 sel_chain=1; do
  timeout -k 10 300 python tools/select_probe.py $v > $O/sel_$v.json 2>&1 || { tail $O/sel_$v.json; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/sel_$v.json').read().strip().splitlines()[-1]); print('$v', d['adaptive_percentage']['ms'], d['adaptive_percentage']['kernel_ms'], d['percentage_100']['ms'])"
done
timeout -k 10 600 python tools/dropin_probe.py > $O/dropin.json 2> $O/dropin.err || { tail $O/dropin.err; exit 1; }
cut -c1-1500 $O/dropin.json
for o in "k2l_co_t=0" "k2l_co_t=1"; do
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 --opt $o > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold.log').read().strip().splitlines()[-1]); print('$o', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'], d['k1']['ms'], d['k1']['frac'])"
done
