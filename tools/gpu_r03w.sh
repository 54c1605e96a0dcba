# selection walk: in-range nodes' A ranks kept in the list (sra), + the select word folded into the
# rank round trip (sr2) vs g4: selection tests on the tree's library (k2c = sr2 + the k2l prefetch
# copied at the loop top), the config-3 queue timed per library; the drop-in leg with the
# branch-free feasible list; hot-value tests on k2c; cold K2 sr2 vs k2c and the option sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash tools/gpu_select_ab.sh r03w g4 sra sr2 || exit 1
timeout -k 10 600 python tools/dropin_probe.py > gpurun_out/r03w/dropin.json 2> gpurun_out/r03w/dropin.err || { tail gpurun_out/r03w/dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03w/dropin.json')); d.pop('workload'); d.get('cpu_same_harness',{}).pop('how',None); print(json.dumps(d)[:1200])"
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hot" > gpurun_out/r03w/pytest_hot.log 2>&1 || { tail -30 gpurun_out/r03w/pytest_hot.log; exit 1; }
tail -1 gpurun_out/r03w/pytest_hot.log
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L gpurun_out/r03w/orig.so
trap 'cp gpurun_out/r03w/orig.so $L' EXIT
for rep in 1 2; do for v in sr2 k2c; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 > gpurun_out/r03w/cold_$v.log 2>&1 || { tail -30 gpurun_out/r03w/cold_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r03w/cold_$v.log').read().strip().splitlines()[-1]); print('$v cold', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'], d['k1']['ms'], d['k1']['frac'], d['k1_records']['ms'], d['k1_records']['frac'])"
done; done
cp gpurun_out/r03w/orig.so $L
timeout -k 10 600 bash tools/gpu_r03v.sh || exit 1
