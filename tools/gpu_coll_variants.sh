# The group's batch form with the collective rehearsed on one device (--group-collective 2): where
# the window's all-reduce time goes.  Variants of dispatch / threads / window, then one kernel trace.
#   bash tools/gpu_coll_variants.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --no-extras --no-cpu-baseline --group-collective 2"
run() {  # name, args
  timeout -k 10 300 $B $2 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['batches_in_flight']['batch_latency_ms'], d['keys_match_stream'], d['host'].get('enqueue_us_per_step'))"
}
run q_caller "--steps 20 --warmup 5"
run streams "--steps 20 --warmup 5 --group-dispatch 0"
run q_workers "--steps 20 --warmup 5 --group-threads 1"
run q_caller100 "--steps 100 --warmup 5"
run q_nocoll "--steps 20 --warmup 5 --group-collective 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o tr \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-cpu-baseline --group-collective 2 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
ls $O/trace
