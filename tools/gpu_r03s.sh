# step pieces gated (prow only when pieces run: producers past 4 rounds and >= 32 pod tiles) (g2)
# vs base (round-2 kernels): parity of the product library, then same-box A/B incl. cold 4M K1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_step.log 2>&1 || { tail -40 $O/pytest_step.log; exit 1; }
tail -1 $O/pytest_step.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 bash tools/gpu_lib_ab.sh r03s_ab base g2 || exit 1
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for v in base g2; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 > $O/cold_$v.log 2>&1 || { tail -30 $O/cold_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold_$v.log').read().strip().splitlines()[-1]); print('$v cold', d['k2']['ms'], d['k2']['frac'], d['k1']['ms'], d['k1']['frac'])"
  timeout -k 10 300 python -u bench.py --config 3 --steps 200 --inflight 1 --no-extras --no-cpu-baseline --no-greedy > $O/b3_$v.log 2>&1 || { tail -30 $O/b3_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/b3_$v.log').read().strip().splitlines()[-1]); print('$v config3 one batch', d['ms_per_step'], d['kernel_ms'])"
done
cp $O/orig.so $L
timeout -k 10 300 python tools/trace_step.py --config 3 --nodes 4000000 --bindings 16000000 > $O/trace4M.json 2> $O/trace4M.err || { tail $O/trace4M.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/trace4M.json'))
for k in ('K1','K3s'):
    if k in d: print(k, d[k]['span'], d[k]['workgroups'], {p:x['med'] for p,x in d[k]['phases'].items()}, {p:x['med'] for p,x in d[k].get('sub',{}).items()})
"
