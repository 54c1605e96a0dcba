# config-4 shard (125k nodes x 100k pods): K3s slices per pod tile (option k3s_blocks = producer
# blocks per workgroup; 0 = the geometry's default, R = 16 here), alone and with middle pieces cut;
# ms per batch one alone / 4 in flight, keys equal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k3; mkdir -p $O
for rep in 1 2; do
for o in "k3s_blocks=0" "k3s_blocks=16" "k3s_blocks=8" "k3s_blocks=64" "k3s_blocks=16 step_pieces=1" "k3s_blocks=8 step_pieces=1"; do
  args=""; for x in $o; do args="$args --opt $x"; done
  timeout -k 10 200 python tools/inflight_probe.py --config 4 --inflight 1,4 --bound $args > $O/inf.json 2>&1 || { tail $O/inf.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/inf.json').read().strip().splitlines()[-1]); print('$o', d['inflight1']['ms_per_step'], d['inflight4']['ms_per_step'], d['inflight4']['keys_equal'], d['inflight1'].get('kernel_ms'))"
done; done
