# Dispatch queues: the kernarg-placement probe, the queue parity tests, then the config-3 step
# through the group on HIP streams vs queues (same box, two rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05aql}
mkdir -p $O
timeout -k 10 120 ./tools/bin_aql_probe > $O/aql_probe.txt 2>&1 || { cat $O/aql_probe.txt; exit 1; }
cat $O/aql_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_aql_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
[ -n "$NOBENCH" ] && exit 0
for rep in 1 2; do
  for d in "0 0" "1 0" "1 1"; do
    set -- $d
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 100 --opt dispatch=$1 --opt dispatch_ring=$2 > $O/b_${1}${2}_$rep.log 2>&1 || { tail -20 $O/b_${1}${2}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${1}${2}_$rep.log').read().strip().splitlines()[-1])
print('dispatch $1 ring $2 rep $rep', d['ms_per_step'], d['value'], d['host'], d['batches_in_flight']['batch_latency_ms'])"
  done
done
