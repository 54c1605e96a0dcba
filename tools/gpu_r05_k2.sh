# K2 change check: hot-value parity tests, then the cold 4M x 16M K2 (ordered and stamp paths) and
# the config-3 step's kernels, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05k2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_step_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --leg cold --steps 5 > $O/cold_$rep.log 2>&1 || { tail -20 $O/cold_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/cold_$rep.log').read().strip().splitlines()[-1])
print('cold rep $rep', 'k2', d['k2']['ms'], d['k2']['kernels'], 'k2ts', d['k2_timestamp_path']['ms'], d['k2_timestamp_path']['kernels'], 'k1', d['k1']['ms'])"
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-cold --no-greedy --steps 100 --warmup 5 > $O/c3_$rep.log 2>&1 || { tail -20 $O/c3_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3_$rep.log').read().strip().splitlines()[-1])
print('config3 rep $rep', d['ms_per_step'], d['kernel_ms'], d['batches_in_flight'].get('batch_latency_ms'))"
done
