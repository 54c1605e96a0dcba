# Large-form K2's second kernel (k2y_bin_hist): how many 16-byte blocks of each region's run
# it loads up front (engine option k2y_first), cold 4M x 16M, both K2 paths, two passes.
#   [F="..."] [X="--opt k2l_hot=1"] bash tools/gpu_k2y.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-k2y}
F=${F:-3 4 5 6 8}   # k2y_first values; X: extra bench arguments
mkdir -p $OUT
for pass in 1 2; do
  for f in $F; do
    timeout -k 10 200 python -u bench.py --leg cold --steps 5 --no-cpu-baseline --opt k2y_first=$f $X \
      > $OUT/p${pass}_f$f.log 2>&1 || { tail -20 $OUT/p${pass}_f$f.log; exit 1; }
    python3 - $OUT/p${pass}_f$f.log "pass $pass k2y_first=$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a, b = d["k2"], d["k2_timestamp_path"]
print(sys.argv[2], "ordered", a["ms"], a["kernels"], "| stamp", b["ms"], b["frac"], b["kernels"])
PY
  done
done
