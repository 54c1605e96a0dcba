# Engine option variants of the config-3 step on dispatch queues (the default group path), 100
# timed batches, same box, two rounds; "-" = defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05qopts}
mkdir -p $O
for rep in 1 2; do
  for v in - k1_threads=128 k2x_threads=1024 k3s_blocks=32 k3s_blocks=128 step_rows=0; do
    a=""; [ "$v" != - ] && a="--opt $v"
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 100 $a > $O/b_${v}_$rep.log 2>&1 || { tail -20 $O/b_${v}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v rep $rep', d['ms_per_step'], 'latency', d['batches_in_flight']['batch_latency_ms'], d['kernel_ms'])"
  done
done
