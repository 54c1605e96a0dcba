# The drop-in's update kernel on the engine's own dispatch queue (engine option update_queue) vs HIP
# on the engine stream: drop-in parity tests, the update-gap probe, then the drop-in harness at
# config 3 (churn x1), both ways, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05updq}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/dropin_files.py $O/files > $O/files.txt 2>&1 || { cat $O/files.txt; exit 1; }
read PP SP PD < <(python3 -c "import ast; print(*ast.literal_eval(open('$O/files.txt').read().strip().splitlines()[-1]))")
for rep in 1 2 3; do
  for m in "" queue; do
    timeout -k 10 120 ./tools/bin_update_gap_probe tests/golden/policy_default.yaml $m > $O/gap_${m:-stream}_$rep.txt 2>&1 || { cat $O/gap_${m:-stream}_$rep.txt; exit 1; }
    echo "gap probe ${m:-stream} rep $rep: $(head -1 $O/gap_${m:-stream}_$rep.txt) | $(grep 'thread started before' $O/gap_${m:-stream}_$rep.txt)"
    opt=""; [ -n "$m" ] && opt="--engine-opt update_queue=1"
    timeout -k 10 300 ./crane-scheduler_amd/lib/dropin_bench $PP $SP $PD --threads 16 --churn 1 $opt > $O/dropin_${m:-stream}_$rep.json 2> $O/dropin_${m:-stream}_$rep.err || { tail $O/dropin_${m:-stream}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/dropin_${m:-stream}_$rep.json').read().strip().splitlines()[-1])
print('dropin ${m:-stream} rep $rep', {k: d[k] for k in d if 'cycle' in k or 'first' in k or 'median' in k}, d.get('matches_engine_chosen'))"
  done
done
