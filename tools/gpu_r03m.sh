set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_plugin_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python tools/dropin_probe.py > $O/dropin.json 2> $O/dropin.err || { tail $O/dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin.json')); d.pop('workload'); d['cpu_same_harness'].pop('how'); print(json.dumps(d))"
