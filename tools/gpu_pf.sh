# Prefetching count pass (k1_count_form 4): step parity tests, then the cold 4M-node leg for the
# fused pass, the split form with the default count pass, and the split form with the prefetching
# one, two rounds on one box.      bash tools/gpu_pf.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pf}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_step.log 2>&1 || { tail -40 $O/pytest_step.log; exit 1; }
tail -1 $O/pytest_step.log
for rep in 1 2; do
  for v in fused split split_pf; do
    case $v in
      fused) OPTS="";;
      split) OPTS="--opt k1_split=1 --opt emit_threads=64";;
      split_pf) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=4";;
    esac
    timeout -k 10 300 python bench.py --leg cold --steps 7 $OPTS > $O/cold_${v}_$rep.json 2> $O/cold_${v}_$rep.err || { tail $O/cold_${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys; c=json.load(open(sys.argv[1])); print(sys.argv[2], 'k1', c['k1']['ms'], c['k1']['frac'], c['k1'].get('kernels'), 'k2', c['k2']['ms'])
" $O/cold_${v}_$rep.json $v
  done
done
