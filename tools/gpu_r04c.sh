# Round 4: the cold 4M-node node pass, fused vs split forms (count pass register budgets,
# one-wave k3a_emit), with K2 on both paths.   bash tools/gpu_r04c.sh <tag> "<variant>;<variant>..."
# a variant: space-separated engine options (name=value), "default" for none
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
IFS=';' read -ra VARS <<< "${2:-default;k1_split=1 emit_threads=64;k1_split=1 emit_threads=64 k1_count_form=1;k1_split=1 emit_threads=64 k1_count_form=2;k1_split=1 emit_threads=64 k1_count_form=3}"
for o in "${VARS[@]}"; do
  args=""; for x in $o; do [ "$x" != default ] && args="$args --opt $x"; done
  f=$OUT/cold_$(echo $o | tr ' =' '__').json
  timeout -k 10 300 python bench.py --leg cold --steps 7 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: (d[k]['ms'], d[k]['frac']) for k in ('k2','k2_timestamp_path','k1','k1_records')}, d['k1'].get('kernels'), d['k2'].get('kernels'))" $f "$o"
done
# phase traces of the node pass at 4M nodes: fused, and the split count pass
for o in "" "--opt k1_split=1 --opt emit_threads=64"; do
  f=$OUT/trace4M_$(echo "$o" | tr ' =-' '___').json
  timeout -k 10 300 python tools/trace_step.py --nodes 4000000 --bindings 16000000 --reps 3 $o > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], json.dumps(d.get('K1'))[:600])" $f "trace $o"
done
