# K1: count/offset words ahead of the SoA stream (hx); K3s: middle pieces cut into elementary
# pieces per block with per-tile ranges (pc = hx + pieces).  Parity of the product library
# (pc), then same-box A/B base / hx / pc (config 3 in flight, config 4, config-4 shard trace,
# cold 4M K1, config 3 one batch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_step_gpu.py tests/test_engine_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 bash tools/gpu_lib_ab.sh r03n_ab base hx pc || exit 1
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for v in base hx pc; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 > $O/cold_$v.log 2>&1 || { tail -30 $O/cold_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold_$v.log').read().strip().splitlines()[-1]); print('$v cold', d['k2']['ms'], d['k2']['frac'], d['k1']['ms'], d['k1']['frac'])"
  timeout -k 10 300 python -u bench.py --config 3 --steps 200 --inflight 1 --no-extras --no-cpu-baseline --no-greedy > $O/b3_$v.log 2>&1 || { tail -30 $O/b3_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/b3_$v.log').read().strip().splitlines()[-1]); print('$v config3 one batch', d['ms_per_step'], d['kernel_ms'])"
done
