# GPU round trip on the box: parity tests, smoke, bench, cold-cache K1/K2 stream bench,
# rocprofv3 kernel stats of the bench.   Usage: bash tools/gpu_verify.sh <tag> [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
fi
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
timeout -k 10 300 python tools/stream_bench.py > $OUT/stream.json 2> $OUT/stream.err || { tail -20 $OUT/stream.err; exit 1; }
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o bench \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-greedy > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
# one batch at a time: the kernels' own durations (what bench.py's kernel_ms / roofline use)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof1 -o bench1 \
    -- python3 $GRAFT_REPO_ROOT/bench.py --inflight 1 --no-cpu-baseline --no-greedy --no-extras > $OUT/prof1.log 2>&1 || { tail -20 $OUT/prof1.log; exit 1; }
tail -3 $OUT/pytest_gpu.log; cat $OUT/smoke.log; tail -1 $OUT/bench.log | cut -c1-3000
python3 tools/kstats.py $OUT/prof/bench_kernel_stats.csv
python3 tools/kstats.py $OUT/prof1/bench1_kernel_stats.csv
