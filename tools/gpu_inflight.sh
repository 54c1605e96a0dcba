# Headline step throughput vs batches in flight (engines x HIP streams), config 3, two rounds.
#   bash tools/gpu_inflight.sh <tag> [K ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-inflight}
shift
KS=${*:-2 3 4 5 6 8}
mkdir -p $O
for rep in 1 2; do
  for k in $KS; do
    timeout -k 10 200 python -u bench.py --no-extras --no-cold --no-cpu-baseline --no-greedy --steps 400 --inflight $k > $O/k${k}_$rep.log 2>&1 || { tail -20 $O/k${k}_$rep.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('inflight', sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), 'M placements/s host', d['host']['enqueue_us_per_step'], 'keys_agree', d['batches_in_flight']['keys_agree'])
" $O/k${k}_$rep.log $k
  done
done
