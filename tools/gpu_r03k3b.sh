# config 3 (100k nodes x 10k pods): K3s slices per pod tile, default (R = 16) vs 64 blocks per
# workgroup (R = 8) vs 48; ms per batch one alone / 4 in flight, keys equal; three passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k3b; mkdir -p $O
for rep in 1 2 3; do
for o in "k3s_blocks=0" "k3s_blocks=64" "k3s_blocks=48"; do
  timeout -k 10 200 python tools/inflight_probe.py --config 3 --inflight 1,4 --bound --opt $o > $O/inf.json 2>&1 || { tail $O/inf.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/inf.json').read().strip().splitlines()[-1]); print('$o', d['inflight1']['ms_per_step'], d['inflight4']['ms_per_step'], d['inflight4']['keys_equal'])"
done; done
