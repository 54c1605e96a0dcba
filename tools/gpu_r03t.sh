# K1 load section back to round 2 (g4 = pieces gated only) vs base: parity of the product library,
# then same-box cold 4M K1 and config-3 in-flight A/B, twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_step_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for rep in 1 2; do
for v in base g4; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 > $O/cold_$v.log 2>&1 || { tail -30 $O/cold_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold_$v.log').read().strip().splitlines()[-1]); print('$v cold', d['k2']['ms'], d['k2']['frac'], d['k1']['ms'], d['k1']['frac'])"
  timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 > $O/inf_$v.json 2>&1 || { tail $O/inf_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/inf_$v.json').read().strip().splitlines()[-1]); print('$v c3 1/4', d['inflight1']['ms_per_step'], d['inflight4']['ms_per_step'])"
done
done
