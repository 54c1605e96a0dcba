# GPU: config-4 shard bench A/B over K3s launch knobs, alternating.  Usage: bash tools/gpu_env_ab_c4.sh <tag> "<ENV=..>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    envs=""; [ "$cfg" != "-" ] && envs="$cfg"
    env $envs timeout -k 10 120 python bench.py --config 4 --no-cpu-baseline --no-greedy --steps 100 --warmup 5 > $OUT/ab_${i}_${rep}.json 2> $OUT/ab_${i}_${rep}.err || { echo "bench failed: $cfg"; tail -5 $OUT/ab_${i}_${rep}.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['stage_ms'])" $OUT/ab_${i}_${rep}.json "$cfg"
  done
done
