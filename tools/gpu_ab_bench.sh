# Same-box A/B of engine builds on the headline: crane-scheduler_amd/lib_ab/lib_<V>.so swapped in
# as the engine library (built by: make -C crane-scheduler_amd/csrc OBJ=_obj_ab/<V>
# LIB=../lib_ab/lib_<V>.so EXTRA="-D..."), per variant the group bench at 100 and 20 batches
# (two rounds, alternating) and the one-batch kernel times.  AB_TESTS=<pytest files>: parity first.
#   bash tools/gpu_ab_bench.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for v in "$@"; do
  if [ -n "$AB_TESTS" ]; then
    cp crane-scheduler_amd/lib_ab/lib_$v.so $L || exit 1
    timeout -k 10 300 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 \
      || { tail -20 $O/pytest_$v.log; exit 1; }
    echo "$v: $(tail -1 $O/pytest_$v.log)"
  fi
done
for rep in 1 2; do
  for v in "$@"; do
    cp crane-scheduler_amd/lib_ab/lib_$v.so $L || exit 1
    for st in 100 20; do
      timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-extras --no-cpu-baseline $AB_ARGS > $O/b_${v}_${st}_$rep.log 2>&1 || { tail -20 $O/b_${v}_${st}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b_${v}_${st}_$rep.log').read().strip().splitlines()[-1])
print('$v', 'steps $st rep $rep:', d['ms_per_step'], 'ms/batch, one batch', d['batches_in_flight']['batch_latency_ms'], 'kernels', d['kernel_ms'], 'keys', d['keys_match_stream'], d['keys_match_oracle_sample'])"
    done
  done
done
