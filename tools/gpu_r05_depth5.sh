# Four vs five batches in flight on dispatch queues (config 3, 200 timed batches), same box, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05d5}
mkdir -p $O
for rep in 1 2 3; do
  for k in 4 5; do
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 200 --inflight $k > $O/b_${k}_$rep.log 2>&1 || { tail -20 $O/b_${k}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${k}_$rep.log').read().strip().splitlines()[-1])
print('inflight $k rep $rep', d['ms_per_step'], 'enqueue', d['host']['enqueue_us_per_step'])"
  done
done
