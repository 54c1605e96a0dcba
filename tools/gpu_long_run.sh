# The headline over long timed regions (thousands of batches): does the per-batch time hold?
# Variants: plain, several enqueuing threads, graph replay.   bash tools/gpu_long_run.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-long}
mkdir -p $OUT
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold "$@" \
    > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  python3 - $OUT/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:24s} {d['ms_per_step']:.4f} ms/batch {d['value']:.4g}/s host {d.get('host')}")
PY
}
for pass in 1 2; do
  run p${pass}_s512 --steps 512 || exit 1
  run p${pass}_s2000 --steps 2000 || exit 1
  run p${pass}_s8000 --steps 8000 || exit 1
  run p${pass}_s8000_t2 --steps 8000 --enqueue-threads 2 || exit 1
  run p${pass}_s8000_t4 --steps 8000 --enqueue-threads 4 || exit 1
  run p${pass}_s8000_graph --steps 8000 --graph || exit 1
done
