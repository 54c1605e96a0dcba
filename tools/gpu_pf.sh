# Split count pass variants: step parity tests, then the cold 4M-node leg for the fused pass, the
# split form with the default count pass, the prefetching one (k1_count_form 4) and the streamed
# one (k1_count_form 5 / 6 / 7: registers for 8 / 7 / 6 waves per SIMD, k3a_emit rebuilding the stepped
# records; 8 / 9: the count pass writing them, 6 / 5 waves), two rounds on one box.
#   bash tools/gpu_pf.sh <tag> [variants...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pf}
shift
VARS=${*:-fused split split_pf split_s5 split_s6 split_s7}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_step.log 2>&1 || { tail -40 $O/pytest_step.log; exit 1; }
tail -1 $O/pytest_step.log
for rep in 1 2; do
  for v in $VARS; do
    case $v in
      fused) OPTS="";;
      split) OPTS="--opt k1_split=1 --opt emit_threads=64";;
      split_pf) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=4";;
      split_s5) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=5";;
      split_s6) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=6";;
      split_s7) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=7";;
      split_s8) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=8";;
      split_s9) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=9";;
      split_s10) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=10";;
      split_s11) OPTS="--opt k1_split=1 --opt emit_threads=64 --opt k1_count_form=11";;
    esac
    timeout -k 10 300 python bench.py --leg cold --steps 7 $OPTS > $O/cold_${v}_$rep.json 2> $O/cold_${v}_$rep.err || { tail $O/cold_${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys; c=json.load(open(sys.argv[1])); print(sys.argv[2], 'k1', c['k1']['ms'], c['k1']['frac'], c['k1'].get('kernels'), 'k2', c['k2']['ms'])
" $O/cold_${v}_$rep.json $v
  done
done
