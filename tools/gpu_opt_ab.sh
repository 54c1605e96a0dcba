# Same-box A/B of engine options on the headline group bench: each variant is a space-separated
# list of name=value engine options ("-" = defaults; a word starting with -- is passed to bench.py
# as it is, e.g. --inflight=8), two rounds alternating, 100 and 20 batches.
# AB_TESTS=<pytest args>: run first.  AB_ARGS: extra bench.py arguments for every run.
#   bash tools/gpu_opt_ab.sh <tag> "-" "k2_delta=0" "k2_delta=0 k1_stream=0" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
  echo "tests: $(tail -1 $O/pytest.log)"
fi
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1)); a=""
    if [ "$v" != "-" ]; then for o in $v; do case $o in --*) a="$a $o";; *) a="$a --opt $o";; esac; done; fi
    for st in 100 20; do
      f=$O/b_${i}_${st}_$rep.log
      timeout -k 10 300 python bench.py --steps $st --warmup ${AB_WARMUP:-16} --no-extras --no-cpu-baseline $a $AB_ARGS > $f 2>&1 || { tail -20 $f; exit 1; }
      python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('[$v]', 'steps $st rep $rep:', d['ms_per_step'], 'ms/batch, one batch', d['batches_in_flight']['batch_latency_ms'], 'kernels', d['kernel_ms'], 'keys', d['keys_match_stream'], d['keys_match_oracle_sample'])"
    done
  done
done
