# Host enqueue cost per step by bench path: group vs ranks (one GPU), advancing vs fixed batch times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05h}
mkdir -p $O
for v in "group 1" "group 6" "ranks 1" "ranks 6"; do
  set -- $v
  timeout -k 10 120 python bench.py --engine $1 --now-cycle $2 --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-greedy > $O/$1_$2.log 2>&1 || { tail -20 $O/$1_$2.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/$1_$2.log').read().strip().splitlines()[-1])
print('$1 cycle $2', d['ms_per_step'], d['host']['enqueue_us_per_step'], d['batches_in_flight']['batch_latency_ms'], d['kernel_ms'])"
done
