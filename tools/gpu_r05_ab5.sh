# Same-box A/B of engine builds through the group on dispatch queues (bench.py, config 3):
# crane-scheduler_amd/lib_ab/lib_<V>.so swapped in; parity tests on the first variant; then per
# round and variant the default-count (100) and the driver's 20-batch timed regions.
#   AB_TESTS="tests/..." bash tools/gpu_r05_ab5.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
if [ -n "$AB_TESTS" ]; then
  for v in "$@"; do
    cp crane-scheduler_amd/lib_ab/lib_$v.so $L || exit 1
    timeout -k 10 400 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
    echo "$v: $(tail -1 $O/pytest_$v.log)"
  done
fi
for rep in 1 2; do
  for steps in 100 20; do
    for v in "$@"; do
      cp crane-scheduler_amd/lib_ab/lib_$v.so $L || exit 1
      w=3; [ $steps = 20 ] && w=5
      timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps $steps --warmup $w > $O/b_${v}_${steps}_$rep.log 2>&1 || { tail -20 $O/b_${v}_${steps}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b_${v}_${steps}_$rep.log').read().strip().splitlines()[-1])
print('$v steps $steps rep $rep', d['ms_per_step'], round(d['value']/1e6,1), 'M/s enqueue', d['host']['enqueue_us_per_step'], 'latency', d['batches_in_flight']['batch_latency_ms'], 'k3s', d['kernel_ms'].get('k3s_eval'))"
    done
  done
done
