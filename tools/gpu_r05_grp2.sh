# Group tests, then the 20- and 100-batch step on the group vs the ranks path, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05grp2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_group_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--no-extras --no-cpu-baseline --no-cold --no-greedy"
for rep in 1 2; do
  for st in 20 100; do
    for e in group ranks; do
      n=${e}_${st}_$rep
      timeout -k 10 200 python bench.py $B --steps $st --warmup 5 --engine $e > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], d['batches_in_flight'].get('batch_latency_ms'), d['host'].get('enqueue_us_per_step'))"
    done
  done
done
