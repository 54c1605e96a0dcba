# K2 form A/B at config 3 (one batch): phase traces and the bench's kernel times per form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/k2f; mkdir -p $O
for f in 0 1 2; do
  timeout -k 10 200 python tools/trace_step.py --config 3 --opt k2_form=$f > $O/trace_$f.json 2> $O/trace_$f.err || { tail $O/trace_$f.err; exit 1; }
done
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 > $O/inf0.json 2>&1 || { tail $O/inf0.json; exit 1; }
timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --opt k2_form=2 > $O/inf2.json 2>&1 || { tail $O/inf2.json; exit 1; }
cat $O/inf0.json $O/inf2.json
