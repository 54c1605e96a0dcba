# GPU: parity tests, smoke, bench, rocprof kernel stats, K3 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_$TAG -o bench \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 1
timeout -k 10 600 python tools/k3_ab.py > $OUT/k3_ab.json 2> $OUT/k3_ab.err
