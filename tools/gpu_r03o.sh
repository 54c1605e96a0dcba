# step_pieces with the rank + coverage in one pass (pc2) vs the atomics form (pc) and base:
# parity of the product library, then same-box A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 bash tools/gpu_lib_ab.sh r03o_ab base pc pc2 || exit 1
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for v in base pc2; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 > $O/cold_$v.log 2>&1 || { tail -30 $O/cold_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold_$v.log').read().strip().splitlines()[-1]); print('$v cold', d['k2']['ms'], d['k2']['frac'], d['k1']['ms'], d['k1']['frac'])"
done
python3 - <<'PY'
import json
for v in ('base','pc','pc2'):
    d=json.load(open(f'gpurun_out/r03o_ab/t4_{v}.json'))
    for k in ('K1','K3s'):
        print(v,k, d[k]['span'], {p:x['med'] for p,x in d[k]['phases'].items()})
PY
