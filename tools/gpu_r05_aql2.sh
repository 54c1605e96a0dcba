# Config-3 step through the group: batches in flight (slots) x dispatch (0 HIP streams, 1 queues),
# same box, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05aql2}
mkdir -p $O
for rep in 1 2; do
  for k in 4 6 8 12; do
    for d in 0 1; do
      timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 200 --inflight $k --group-dispatch $d > $O/b_${k}_${d}_$rep.log 2>&1 || { tail -20 $O/b_${k}_${d}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b_${k}_${d}_$rep.log').read().strip().splitlines()[-1])
print('inflight $k dispatch $d rep $rep', d['ms_per_step'], round(d['value']/1e6,1), 'M/s enqueue', d['host']['enqueue_us_per_step'], 'latency', d['batches_in_flight']['batch_latency_ms'])"
    done
  done
done
