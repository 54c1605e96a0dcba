# rocprofv3 PMC passes over a short bench (one counter group per pass, --pmc only,
# no trace domains; FETCH_SIZE and WRITE_SIZE cannot share a pass).  Stops on any
# fault/timeout exit code.  Usage: bash tools/gpu_pmc.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-greedy"
run() {  # name counters...
    local name=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o $name -- $CMD > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc" >> $OUT/status.txt
    case $rc in 124|134|137|139) exit $rc;; esac
    return 0
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run valu SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run l2 TCC_HIT_sum TCC_MISS_sum
python3 tools/pmc_summary.py $OUT > $OUT/summary.json
exit 0
