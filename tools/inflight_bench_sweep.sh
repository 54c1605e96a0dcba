set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/inf; mkdir -p $O
for k in 4 6 8; do
  timeout -k 10 200 python bench.py --inflight $k --no-cpu-baseline --no-greedy --no-extras > $O/b$k.log 2>&1 || { tail $O/b$k.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b$k.log').read().strip().splitlines()[-1]); print($k, d['ms_per_step'], d['batches_in_flight']['batch_latency_ms'], d['kernel_ms'])"
done
