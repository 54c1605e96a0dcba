# Step tests, then the cold 4M K1 with the streamed pass's tail on one wave (k1_tail 0 = auto:
# one wave at this grid) vs on four (4) vs the fused pass, same box, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05k1b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_step_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for f in "k1_tail=0" "k1_tail=4" "k1_stream=0"; do
    timeout -k 10 200 python -u bench.py --leg cold --steps 5 --opt $f > $O/cold_${f}_$rep.log 2>&1 || { tail -20 $O/cold_${f}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/cold_${f}_$rep.log').read().strip().splitlines()[-1])
print('$f rep $rep', 'k1', d['k1']['ms'], d['k1']['frac'])"
  done
done
