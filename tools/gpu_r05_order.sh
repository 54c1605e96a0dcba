# Headline ms per batch and host enqueue vs the legs the bench line carries (same box, two rounds):
# full = the default line; nodropin = minus the drop-in / CPU-baseline / cold / greedy legs;
# bare = --no-extras as well (the headline step alone).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05order}; shift
mkdir -p $O
for rep in 1 2; do
  for v in ${VARIANTS:-full nodropin bare}; do
    a=""; [ $v = nodropin ] && a="--no-cpu-baseline --no-cold --no-greedy"
    [ $v = bare ] && a="--no-cpu-baseline --no-cold --no-greedy --no-extras"
    timeout -k 10 400 python -u bench.py --steps 100 $a "$@" > $O/${v}_$rep.log 2>&1 || { tail -20 $O/${v}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_$rep.log').read().strip().splitlines()[-1])
print('$v', $rep, d['ms_per_step'], d['host'], d['batches_in_flight']['batch_latency_ms'])"
  done
done
