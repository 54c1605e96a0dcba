# K3s slice count (R) sweep at config 3 and 4: stage times per setting
cd "$GRAFT_REPO_ROOT"
for b in 10 40 160 640; do
  echo "blocks=$b"
  CRANE_K3S_BLOCKS=$b timeout -k 10 120 python bench.py --no-cpu-baseline --no-greedy --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stage_ms'])" || exit 1
done
