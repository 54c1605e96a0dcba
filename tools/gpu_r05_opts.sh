# Config-3 step over 20 and 100 timed batches with engine option variants, same box, two rounds.
# Usage: bash tools/gpu_r05_opts.sh <tag> "name=value[,name=value]" ...   ("-" = defaults)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
B="--no-extras --no-cpu-baseline --no-cold --no-greedy"
for rep in 1 2; do
  for v in "$@"; do
    o=""; [ "$v" != "-" ] && for kv in $(echo $v | tr ',' ' '); do o="$o --opt $kv"; done
    for st in 20 100; do
      n=$(echo "${v}_${st}_$rep" | tr '=,' '__')
      timeout -k 10 200 python bench.py $B --steps $st --warmup 5 $o > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1])
print('$v', $st, 'rep $rep', d['ms_per_step'], d['batches_in_flight'].get('batch_latency_ms'), d['kernel_ms'])"
    done
  done
done
