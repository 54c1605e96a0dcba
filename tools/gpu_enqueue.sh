# Headline step with 1 / 2 / 4 host threads enqueuing (4 and 8 batches in flight), config 3,
# 400 batches, two rounds.      bash tools/gpu_enqueue.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-enq}
mkdir -p $O
for rep in 1 2; do
  for v in "4 1" "4 2" "4 4" "8 2" "8 4"; do
    set -- $v
    timeout -k 10 200 python -u bench.py --no-extras --no-cold --no-cpu-baseline --no-greedy --steps 400 --inflight $1 --enqueue-threads $2 > $O/k$1_t$2_$rep.log 2>&1 || { tail -20 $O/k$1_t$2_$rep.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('inflight', sys.argv[2], 'threads', sys.argv[3], d['ms_per_step'], round(d['value']/1e6,1), 'M placements/s host', d['host'], 'keys_agree', d['batches_in_flight']['keys_agree'])
" $O/k$1_t$2_$rep.log $1 $2
  done
done
