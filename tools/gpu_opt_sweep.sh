# Headline (config 3, 4 batches in flight, 512 batches) under engine option variants, two
# interleaved passes on one box, to re-check round-3 defaults against this round's kernels.
#   bash tools/gpu_opt_sweep.sh <tag> "<variant>;<variant>;..."   (variant: "name=value name=value", or "default")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-optsweep}
mkdir -p $OUT
IFS=';' read -ra VARS <<< "$2"
for pass in 1 2; do
  for v in "${VARS[@]}"; do
    opts=""
    [ "$v" != "default" ] && for o in $v; do opts="$opts --opt $o"; done
    name=$(echo "$v" | tr ' =' '_-')
    timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 512 $opts \
      > $OUT/p${pass}_$name.log 2>&1 || { tail -20 $OUT/p${pass}_$name.log; exit 1; }
    python3 - $OUT/p${pass}_$name.log "pass $pass $v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms/batch {d['value']:.4g}/s  one batch {d['kernel_ms']}")
PY
  done
done
