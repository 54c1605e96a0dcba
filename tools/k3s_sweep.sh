# K3s slicing sweep (engine option k3s_blocks) on configs 3 and 4: span per kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
for c in 3 4; do for b in 8 16 32 64; do
  timeout -k 10 120 python tools/trace_step.py --config $c --opt k3s_blocks=$b > $OUT/t${c}_$b.json || exit 1
done; done
