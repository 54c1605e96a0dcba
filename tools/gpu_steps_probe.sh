# How the headline depends on the timed region's length and the warmup (the driver runs
# --steps 20 --warmup 5): ms per batch for several (steps, warmup) pairs, two passes.
#   [X="extra bench args"] bash tools/gpu_steps_probe.sh <tag>
# (run steps2 used a trial bench.py with --settle-ms / --block-sync, since dropped: profiles/r04/short_timed_region.txt)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-steps}
mkdir -p $OUT
for pass in 1 2; do
  for sw in "20 5" "20 200" "100 3" "512 3"; do
    set -- $sw
    timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps $1 --warmup $2 $X \
      > $OUT/p${pass}_s$1_w$2.log 2>&1 || { tail -20 $OUT/p${pass}_s$1_w$2.log; exit 1; }
    python3 - $OUT/p${pass}_s$1_w$2.log "pass $pass steps $1 warmup $2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:32s} {d['ms_per_step']:.4f} ms/batch {d['value']:.4g}/s host {d.get('host')}")
PY
  done
done
