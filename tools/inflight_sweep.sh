# In-flight throughput under engine option variants (tools/inflight_probe.py), config 3.
#   bash tools/inflight_sweep.sh <tag> "<opt> <opt> ..." (each opt: name=value, one run each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 > $OUT/base.json || exit 1
for o in $2; do
  timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --opt $o > $OUT/$o.json || exit 1
done
