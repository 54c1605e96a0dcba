# Cold 4M-node K1: the streamed step pass (k1_stream 1) vs the record-holding fused pass (0), same
# box, interleaved; then the per-workgroup phase traces of both at 4M nodes x 16M bindings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05k1}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py tests/test_engine_gpu.py tests/test_dropin_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
FORMS=${2:-"1 0"}
for rep in 1 2; do
  for f in $FORMS; do
    timeout -k 10 200 python -u bench.py --leg cold --steps 5 --opt k1_stream=$f > $O/cold_${f}_$rep.log 2>&1 || { tail -20 $O/cold_${f}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/cold_${f}_$rep.log').read().strip().splitlines()[-1])
print('k1_stream=$f rep $rep', 'k1', d['k1']['ms'], d['k1']['frac'], 'k2', d['k2']['kernels'], 'k2ts', d['k2_timestamp_path']['kernels'])"
  done
done
for f in $FORMS; do
  timeout -k 10 200 python -u tools/trace_step.py --config 3 --nodes 4000000 --bindings 16000000 --reps 3 --opt k1_stream=$f > $O/trace_$f.json 2>$O/trace_$f.err || { tail -20 $O/trace_$f.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/trace_$f.json')); k=d['K1']; print('trace k1_stream=$f', k['span'], k['phases'], k.get('sub'))"
done
