# Same-box cold 4M K1 time of the ablation builds (tools/k1_ablate_build.sh) swapped in as the
# engine library, two rounds.  Usage: bash tools/gpu_k1_ablate.sh <tag> <mask> ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for rep in 1 2; do
  for m in "$@"; do
    cp crane-scheduler_amd/lib_ab/lib_$m.so $L || exit 1
    timeout -k 10 200 python -u bench.py --leg cold --steps 5 > $O/cold_${m}_$rep.log 2>&1 || { tail -20 $O/cold_${m}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/cold_${m}_$rep.log').read().strip().splitlines()[-1])
print('$m rep $rep', 'k1', d['k1']['ms'], d['k1']['frac'])"
  done
done
