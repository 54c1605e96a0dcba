# Dispatch queues: a step's first / last packet fenced at system scope (lib_sys) vs agent scope
# (lib_agent), against HIP streams, 100 and 20 timed batches, same box, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05aql3}
mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
cp crane-scheduler_amd/lib_ab/lib_agent.so $L
timeout -k 10 300 python -u -m pytest tests/test_aql_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_agent.log 2>&1 || { tail -30 $O/pytest_agent.log; exit 1; }
echo "agent: $(tail -1 $O/pytest_agent.log)"
for rep in 1 2; do
  for steps in 100 20; do
    for v in "sys 0" "sys 1" "agent 1"; do
      set -- $v
      cp crane-scheduler_amd/lib_ab/lib_$1.so $L
      w=3; [ $steps = 20 ] && w=5
      timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps $steps --warmup $w --group-dispatch $2 > $O/b_$1_$2_${steps}_$rep.log 2>&1 || { tail -20 $O/b_$1_$2_${steps}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b_$1_$2_${steps}_$rep.log').read().strip().splitlines()[-1])
print('$1 dispatch $2 steps $steps rep $rep', d['ms_per_step'], round(d['value']/1e6,1), 'M/s enqueue', d['host']['enqueue_us_per_step'], 'latency', d['batches_in_flight']['batch_latency_ms'])"
    done
  done
done
