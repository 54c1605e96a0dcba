# Dispatch queues and HIP's own hardware queues: batches in flight (one AQL queue per slot) with
# HIP limited to one hardware queue (GPU_MAX_HW_QUEUES=1) vs HIP's default (4), same box, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05hwq}
mkdir -p $O
for rep in 1 2; do
  for hq in 4 1; do
    for k in 4 6 8; do
      GPU_MAX_HW_QUEUES=$hq timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 200 --inflight $k > $O/b_${hq}_${k}_$rep.log 2>&1 || { tail -20 $O/b_${hq}_${k}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b_${hq}_${k}_$rep.log').read().strip().splitlines()[-1])
print('hip queues $hq inflight $k rep $rep', d['ms_per_step'], round(d['value']/1e6,1), 'M/s enqueue', d['host']['enqueue_us_per_step'], 'latency', d['batches_in_flight']['batch_latency_ms'])"
    done
  done
done
