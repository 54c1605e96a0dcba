# GPU: K3s grid-size A/B (CRANE_K3S_BLOCKS) on configs 3 and 4, alternating.
# Usage: bash tools/gpu_k3s_ab.sh <tag> <blocks>...   ("-" = default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
shift
mkdir -p $OUT
for rep in 1 2; do
  for cfg in 3 4; do
    for b in "$@"; do
      envs=""; [ "$b" != "-" ] && envs="CRANE_K3S_BLOCKS=$b"
      env $envs timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-greedy --steps 100 --warmup 10 > $OUT/c${cfg}_$b.json 2> $OUT/c${cfg}_$b.err || { tail -5 $OUT/c${cfg}_$b.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('config', sys.argv[2], 'blocks', sys.argv[3], d['ms_per_step'], d['stage_ms'])" $OUT/c${cfg}_$b.json $cfg "$b"
    done
  done
done
