# The driver's short timed region (--steps 20 --warmup 5): one vs four enqueuing threads, three passes
# (a trial bench.py also had a clock-settle phase and event polling before each wait: both slower,
# profiles/r04/short_timed_region.txt).
#   bash tools/gpu_short_run.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-short}
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
for pass in 1 2 3; do
  run p${pass}_t1 --steps 20 --warmup 5 || exit 1
  run p${pass}_t4 --steps 20 --warmup 5 --enqueue-threads 4 || exit 1
  run p${pass}_t4_100 --steps 100 --warmup 5 --enqueue-threads 4 || exit 1
done
