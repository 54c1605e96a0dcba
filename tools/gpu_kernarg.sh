# Host enqueue cost vs where the HIP runtime puts kernel arguments (HIP_FORCE_DEV_KERNARG, a
# per-process runtime setting): the driver's 20-batch region and a 512-batch one, three passes.
#   bash tools/gpu_kernarg.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-kernarg}
mkdir -p $OUT
run() {  # name, env assignment, bench args...
  local name=$1 envv=$2; shift 2
  env $envv timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold "$@" \
    > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  python3 - $OUT/$name.log "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:24s} {d['ms_per_step']:.4f} ms/batch {d['value']:.4g}/s one batch {d['kernel_ms']} latency {d['batches_in_flight']['batch_latency_ms']} host {d.get('host')}")
PY
}
for pass in 1 2 3; do
  for kv in unset 0 1; do
    e="X=1"; [ $kv != unset ] && e="HIP_FORCE_DEV_KERNARG=$kv"
    run p${pass}_k${kv}_s20 $e --steps 20 --warmup 5 || exit 1
    run p${pass}_k${kv}_s512 $e --steps 512 --warmup 5 || exit 1
  done
done
