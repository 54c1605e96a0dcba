# Round 4 (session 2): GPU suite + smoke + default bench line, then the collective path
# rehearsed on one rank against the same step without it, then a
# kernel + HIP-runtime trace of the rehearsal.        bash tools/gpu_r04s.sh <tag> [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04s}
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-1500
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
for s in 100 512; do
  for rep in 1 2; do
    timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps $s > $OUT/nocoll_${s}_$rep.log 2>&1 || { tail -20 $OUT/nocoll_${s}_$rep.log; exit 1; }
    timeout -k 10 200 python -u bench.py --rehearse-collective --no-extras --no-cpu-baseline --no-greedy --no-cold --steps $s > $OUT/coll_${s}_$rep.log 2>&1 || { tail -20 $OUT/coll_${s}_$rep.log; exit 1; }
    python3 - $OUT $s $rep <<'PY'
import json, sys
o, s, r = sys.argv[1:]
a = json.loads(open(f"{o}/nocoll_{s}_{r}.log").read().strip().splitlines()[-1])
b = json.loads(open(f"{o}/coll_{s}_{r}.log").read().strip().splitlines()[-1])
print(f"steps {s} rep {r}: no collective {a['ms_per_step']} ms/batch, rehearsed {b['ms_per_step']} ({b['ms_per_step'] / a['ms_per_step']:.3f}x), "
      f"all-reduce {b.get('allreduce_ms')} ms/call, keys_match_1gpu {b.get('keys_match_1gpu')}")
PY
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_coll -o coll \
    -- python3 $GRAFT_REPO_ROOT/bench.py --rehearse-collective --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 512 > $OUT/trace_coll.log 2>&1 || { tail -20 $OUT/trace_coll.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_nocoll -o nocoll \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-cpu-baseline --no-greedy --no-cold --steps 512 > $OUT/trace_nocoll.log 2>&1 || { tail -20 $OUT/trace_nocoll.log; exit 1; }
ls -la $OUT/trace_coll $OUT/trace_nocoll
