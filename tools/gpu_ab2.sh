# A/B of step-path settings on the bench (no CPU baseline / greedy): one line per setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
for s in "CRANE_K1_FUSE=1" "CRANE_K1_FUSE=0" "CRANE_K3S_BLOCKS=128" "CRANE_K3S_BLOCKS=256" "CRANE_K3S_BLOCKS=512"; do
  env $s timeout -k 10 120 python bench.py --no-cpu-baseline --no-greedy > $OUT/ab_$s.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['stage_ms'])" $OUT/ab_$s.log "$s"
done
for s in "CRANE_K3S_BLOCKS=256" "CRANE_K3S_BLOCKS=1024"; do
  env $s timeout -k 10 200 python bench.py --config 4 --steps 10 --no-cpu-baseline --no-greedy > $OUT/ab4_$s.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg4', sys.argv[2], d['ms_per_step'], d['stage_ms'])" $OUT/ab4_$s.log "$s"
done
