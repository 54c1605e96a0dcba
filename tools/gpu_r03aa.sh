# host enqueue cost of the step: plain kernel launches when not timing (pl) vs the ext launch
# (fin = the committed build), and pl without the caller-stream completion events (measurement
# only); VARIANTS="fin ev" compares the committed build with the device-synchronize form; config 3, bound step calls, one batch and 4 in flight, three passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03aa; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for rep in 1 2 3; do for v in ${VARIANTS:-fin pl "pl busy_events=0"}; do
  set -- $v
  cp crane-scheduler_amd/lib_ab/lib_$1.so $L
  opt=""; [ -n "$2" ] && opt="--opt $2"
  timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --bound $opt > $O/inf.json 2>&1 || { tail $O/inf.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/inf.json').read().strip().splitlines()[-1]); print('$v', 'one', d['inflight1']['ms_per_step'], d['inflight1']['host_enqueue_ms_per_step'], 'four', d['inflight4']['ms_per_step'], d['inflight4']['host_enqueue_ms_per_step'], d['inflight4']['keys_equal'])"
done; done
