# GPU: parity tests, then the config-3 bench (twice) and the 4M-node cold stream bench.
# Usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-greedy --steps 200 --warmup 10 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { tail -5 $OUT/bench_$rep.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stage_ms'])" $OUT/bench_$rep.json
done
timeout -k 10 300 python tools/stream_bench.py --k2 binned --reps 3 > $OUT/stream.json 2> $OUT/stream.err || { tail -5 $OUT/stream.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps(d['by_k2_mode']['binned']))" $OUT/stream.json
