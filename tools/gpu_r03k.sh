set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_select.py tests/test_plugin_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/select_probe.py > $O/sel.json 2>&1 || { tail $O/sel.json; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/sel.json').read().strip().splitlines()[-1]); print(d['adaptive_percentage']['ms'], d['adaptive_percentage']['kernel_ms'], d['percentage_100']['ms'])"
timeout -k 10 600 python tools/dropin_probe.py > $O/dropin.json 2> $O/dropin.err || { tail $O/dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin.json')); d.pop('workload'); print(json.dumps(d))"
timeout -k 10 300 python -u bench.py --config 3 --steps 100 --no-extras --no-cpu-baseline --no-greedy > $O/b3.log 2>&1 || { tail -30 $O/b3.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b3.log').read().strip().splitlines()[-1]); print('config3', d['ms_per_step'], d['batches_in_flight']['batch_latency_ms'], d['kernel_ms'])"
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 300 python -u bench.py --config 3 --steps 100 --rehearse-collective --no-extras --no-cpu-baseline --no-greedy > $O/r3.log 2>&1 || { tail -30 $O/r3.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/r3.log').read().strip().splitlines()[-1]); print('rehearse3', d['ms_per_step'], d['allreduce_ms'], d['keys_match_1gpu'])"
