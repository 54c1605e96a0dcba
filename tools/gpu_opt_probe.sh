# One engine option A/B at config 3: in-flight probe (1 and 4 batches) and phase trace.
#   bash tools/gpu_opt_probe.sh <tag> <name=value> [<name=value> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
for o in "$@"; do
  timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --opt $o > $O/inf_$o.json 2>&1 || { tail $O/inf_$o.json; exit 1; }
  timeout -k 10 200 python tools/trace_step.py --config 3 --opt $o > $O/trace_$o.json 2> $O/trace_$o.err || { tail $O/trace_$o.err; exit 1; }
  tail -1 $O/inf_$o.json
done
