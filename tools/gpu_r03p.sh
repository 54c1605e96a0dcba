# full GPU suite on the product library (K1 loads ahead, step_pieces gated by producer rounds, plugin
# keyed by Name address); config 3 / 4 bench lines; drop-in leg; K1 phase trace at 4M nodes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --no-greedy --no-extras > $O/b4.log 2>&1 || { tail -30 $O/b4.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b4.log').read().strip().splitlines()[-1]); print('config4', d['ms_per_step'], d['batches_in_flight']['batch_latency_ms'], d['kernel_ms'])"
timeout -k 10 600 python tools/dropin_probe.py > $O/dropin.json 2> $O/dropin.err || { tail $O/dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin.json')); d.pop('workload'); d.get('cpu_same_harness',{}).pop('how',None); print(json.dumps(d)[:1500])"
timeout -k 10 300 python tools/trace_step.py --config 3 --nodes 4000000 --bindings 16000000 > $O/trace4M.json 2> $O/trace4M.err || { tail $O/trace4M.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/trace4M.json'))
for k in ('K2x','K1','K3s'):
    if k in d: print(k, d[k]['span'], d[k]['workgroups'], {p:x['med'] for p,x in d[k]['phases'].items()}, {p:x['med'] for p,x in d[k].get('sub',{}).items()})
"
