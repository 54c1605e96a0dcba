# drop-in cycle: the harness pool before (condition-variable wake per fan-out) and after
# (spin, then sleep), same box, alternating; then the GPU tests that drive the harness
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03dp; mkdir -p $O
L=crane-scheduler_amd/lib
trap 'cp $L/dropin_bench_new $L/dropin_bench' EXIT
for v in old new old new; do
  cp $L/dropin_bench_$v $L/dropin_bench
  timeout -k 10 300 python tools/dropin_probe.py > $O/dp_$v.json 2> $O/dp_$v.err || { tail $O/dp_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/dp_$v.json').read().strip().splitlines()[-1]); d.pop('workload', None); print('$v', json.dumps(d)[:600])"
done
cp $L/dropin_bench_new $L/dropin_bench
timeout -k 10 300 python -u -m pytest tests -m gpu -k "dropin or plugin" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc $?"; tail -1 $O/pytest.log
