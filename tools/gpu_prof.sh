# GPU: rocprofv3 kernel stats of the bench.  Usage: bash tools/gpu_prof.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-p}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o bench \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
python3 tools/kstats.py $OUT/prof/bench_kernel_stats.csv
