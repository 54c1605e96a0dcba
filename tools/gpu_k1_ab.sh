# GPU: cold-cache large-N node pass under env variants and node counts.
# Usage: bash tools/gpu_k1_ab.sh <tag> [nodes...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
shift
mkdir -p $OUT
i=0
for nodes in ${@:-4000000}; do
  for cfg in "-" "CRANE_K1_THREADS=128" "CRANE_K1_KEEP_REC=1"; do
    i=$((i+1)); envs=""; [ "$cfg" != "-" ] && envs="$cfg"
    env $envs timeout -k 10 300 python tools/stream_bench.py --nodes $nodes --k2 binned --reps 3 > $OUT/k1_$i.json 2> $OUT/k1_$i.err || { tail -5 $OUT/k1_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], json.dumps(d['by_k2_mode']['binned']))" $OUT/k1_$i.json "$nodes" "$cfg"
  done
done
