# Round 4: where the rehearsed collective's per-batch cost goes, and hardware queues.
#   bash tools/gpu_r04b.sh <tag>
# 1) config-3 bench without extras: the plain path, the collective rehearsed on one rank
#    (torch.distributed with RCCL initialised, one all-reduce per 64 batches), and the
#    process with RCCL initialised but no collective issued; GPU_MAX_HW_QUEUES 4 (HIP's
#    default) and 8.   2) rocprofv3 kernel + HIP runtime trace of the rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04b}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
run() {  # label, env, args
  local lab=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$lab.json 2> $OUT/$lab.err || { tail -20 $OUT/$lab.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['batches_in_flight']['batch_latency_ms'], d.get('allreduce_ms'), d.get('keys_match_1gpu'))" $OUT/$lab.json $lab
}
# host enqueue: one thread vs one host thread per engine (ctypes drops the GIL in the call)
for q in 4 8; do
  timeout -k 10 240 env GPU_MAX_HW_QUEUES=$q python tools/inflight_probe.py --bound --steps 2000 --inflight 4,8 > $OUT/enq_q$q.json 2>$OUT/enq_q$q.err || { tail -5 $OUT/enq_q$q.err; exit 1; }
  timeout -k 10 240 env GPU_MAX_HW_QUEUES=$q python tools/inflight_probe.py --bound --threads --steps 2000 --inflight 4,8 > $OUT/enq_thr_q$q.json 2>$OUT/enq_thr_q$q.err || { tail -5 $OUT/enq_thr_q$q.err; exit 1; }
  echo "q$q one-thread $(cat $OUT/enq_q$q.json)"; echo "q$q threads $(cat $OUT/enq_thr_q$q.json)"
done
# batches in flight beyond the 4 hardware queues
for k in 6 8; do
  run plain_q8_k$k GPU_MAX_HW_QUEUES=8 python bench.py --no-extras --no-cpu-baseline --steps 512 --inflight $k || exit 1
  run plain_q4_k$k GPU_MAX_HW_QUEUES=4 python bench.py --no-extras --no-cpu-baseline --steps 512 --inflight $k || exit 1
done
for q in 4 8; do
  for rep in 1 2; do
    run plain_q${q}_$rep GPU_MAX_HW_QUEUES=$q python bench.py --no-extras --no-cpu-baseline --steps 512 || exit 1
    run rehearse_q${q}_$rep GPU_MAX_HW_QUEUES=$q python bench.py --no-extras --no-cpu-baseline --steps 512 --rehearse-collective || exit 1
    run rehearse_noar_q${q}_$rep GPU_MAX_HW_QUEUES=$q python bench.py --no-extras --no-cpu-baseline --steps 512 --rehearse-collective --ar-group 512 || exit 1
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_rehearse -o reh \
  -- python3 bench.py --no-extras --no-cpu-baseline --steps 512 --rehearse-collective > $OUT/trace_rehearse.log 2>&1 || { tail -20 $OUT/trace_rehearse.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_plain -o plain \
  -- python3 bench.py --no-extras --no-cpu-baseline --steps 512 > $OUT/trace_plain.log 2>&1 || { tail -20 $OUT/trace_plain.log; exit 1; }
ls -R $OUT | head -40
