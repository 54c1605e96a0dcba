# Interleaved dispatch queues (group dispatch 2: two slots' steps side by side per queue): parity
# tests, then the config-3 step at 4 / 6 / 8 slots vs one queue per slot (dispatch 1, 4 slots) and
# HIP streams (dispatch 0), 100 and 20 batches, same box, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05aql4}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_aql_gpu.py tests/test_group_gpu.py -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for steps in 100 20; do
    for v in "0 4" "1 4" "2 6" "2 8"; do
      set -- $v
      w=3; [ $steps = 20 ] && w=5
      timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps $steps --warmup $w --group-dispatch $1 --inflight $2 > $O/b_$1_$2_${steps}_$rep.log 2>&1 || { tail -20 $O/b_$1_$2_${steps}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b_$1_$2_${steps}_$rep.log').read().strip().splitlines()[-1])
print('dispatch $1 inflight $2 steps $steps rep $rep', d['ms_per_step'], round(d['value']/1e6,1), 'M/s enqueue', d['host']['enqueue_us_per_step'], 'latency', d['batches_in_flight']['batch_latency_ms'])"
    done
  done
done
