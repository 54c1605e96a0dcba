# The step's engine paths on one device, same box, two rounds: the C ABI group (caller thread, no
# collective: the default at one device), the group with a worker thread and the in-library RCCL
# all-reduce rehearsed (collective 2), and the torch.distributed ranks path (with and without its
# rehearsed collective, under torchrun with one rank).  100 and 20 timed batches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05grp}
mkdir -p $O
B="--no-extras --no-cpu-baseline --no-cold --no-greedy"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1])
print('$n', d['steps'], d['ms_per_step'], d['value'], d['host'].get('enqueue_us_per_step'), d['config'].get('engine'))"
}
for rep in 1 2; do
  for st in 100 20; do
    W="--steps $st --warmup 5"
    run grp_${st}_$rep python bench.py $B $W
    run grpcoll_${st}_$rep python bench.py $B $W --group-collective 2 --group-threads 1
    run ranks_${st}_$rep python bench.py $B $W --engine ranks
    run rankscoll_${st}_$rep python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py $B $W --engine ranks --rehearse-collective
  done
done
