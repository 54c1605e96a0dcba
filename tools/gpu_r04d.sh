# Round 4: GPU suite, drop-in leg at 5k / 100k nodes, cold legs (default).   bash tools/gpu_r04d.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/dropin_probe.py 5000 256 > $OUT/dropin_5k.json 2> $OUT/dropin_5k.err || { tail -30 $OUT/dropin_5k.err; exit 1; }
timeout -k 10 400 python -u tools/dropin_probe.py 100000 256 > $OUT/dropin_100k.json 2> $OUT/dropin_100k.err || { tail -30 $OUT/dropin_100k.err; exit 1; }
for f in dropin_5k dropin_100k; do python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['dropin_ms_per_pod'], d['matches_engine_chosen'], d['matches_oracle_sample'], d.get('cpu_same_harness_ms_per_pod'))
for k in ('churn_x1','churn_x10','frozen'): print('  ', k, {x: d[k][x] for x in ('cycle_ms_median','cycle_ms_p90','first_call_ms_median','filter_fanout_ms_median','score_fanout_ms_median','pool_noop_ms_median','patches','nodes_updated')})
" $OUT/$f.json $f; done
bash tools/gpu_r04c.sh ${1:-r04d} "default" || exit 1
