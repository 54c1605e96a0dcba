# The rehearsed collective path's host cost: config 3, 512 batches,
# with and without the collective, under environment variants; each line reports ms per
# batch and the enqueuing thread's wall / CPU us per step and the busiest other threads.
#   bash tools/gpu_coll_probe.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-coll}
mkdir -p $OUT
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
ARGS="--no-extras --no-cpu-baseline --no-greedy --no-cold --steps 512"
run() {  # name, env assignments..., then "--" and extra bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python -u bench.py $ARGS "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  python3 - $OUT/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:28s} {d['ms_per_step']:.4f} ms/batch  host {d.get('host')}")
PY
}
run nocoll X=1 -- || exit 1
run coll X=1 -- --rehearse-collective || exit 1
run coll_hwq8 GPU_MAX_HW_QUEUES=8 -- --rehearse-collective || exit 1
run nocoll_hwq8 GPU_MAX_HW_QUEUES=8 -- || exit 1
run coll_nomon TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 -- --rehearse-collective || exit 1
run coll_eng X=1 -- --rehearse-collective --ar-stream engine || exit 1
run nocoll2 X=1 -- || exit 1
run coll2 X=1 -- --rehearse-collective || exit 1
