# In-flight throughput under engine option variants (tools/inflight_probe.py), config 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 > $OUT/base.json || exit 1
for t in 256 512; do
  timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --opt k2x_threads=$t > $OUT/k2x_$t.json || exit 1
done
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --opt k1_threads=128 > $OUT/k1_128.json || exit 1
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --opt k2x_threads=256 --opt k1_threads=128 > $OUT/both.json || exit 1
