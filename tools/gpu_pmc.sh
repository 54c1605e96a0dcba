# rocprofv3 PMC passes over short bench runs (one counter group per pass, --pmc
# only, no trace domains; FETCH_SIZE and WRITE_SIZE cannot share a pass), one
# summary per workload keyed by the kernel-source hash, so bench.py attaches
# traffic only to lines measured on the same kernels and config:
#   profiles/pmc/config3_<hash>.json   headline step, config 3
#   profiles/pmc/config2_<hash>.json   per-pair matrix leg, config 2
#   profiles/pmc/config3m_<hash>.json  per-pair matrix leg at config 3 size
#   profiles/pmc/config4m_<hash>.json  cold-cache 4M-node pass (tools/stream_bench.py)
#   profiles/pmc/configcold_<hash>.json  bench.py's cold-cache K1/K2 leg (roofline_cold)
# Stops on any fault/timeout exit code.  Usage: bash tools/gpu_pmc.sh <tag> [workloads]
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pmc}
WL=${2:-"3 2 3m"}
export TMPDIR=/tmp
for w in $WL; do
    OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$w
    mkdir -p $OUT
    case $w in
        2) CMD="python3 $GRAFT_REPO_ROOT/bench.py --leg matrix2 --steps 5";;
        3m) CMD="python3 $GRAFT_REPO_ROOT/bench.py --leg matrix3 --steps 3";;
        4m) CMD="python3 $GRAFT_REPO_ROOT/tools/stream_bench.py --k2 auto --reps 2";;
        cold) CMD="python3 $GRAFT_REPO_ROOT/bench.py --leg cold --steps 2";;
        *) CMD="python3 $GRAFT_REPO_ROOT/bench.py --config $w --steps 5 --warmup 1 --inflight 1 --no-cpu-baseline --no-greedy --no-extras";;
    esac
    for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "valu SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "l2 TCC_HIT_sum TCC_MISS_sum" "lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
        set -- $pass
        name=$1; shift
        timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o $name -- $CMD > $OUT/$name.log 2>&1
        rc=$?
        echo "$w $name rc=$rc" >> $OUT/status.txt
        case $rc in 124|134|137|139) exit $rc;; esac
    done
    python3 tools/pmc_summary.py $OUT --config $w > $OUT/summary.json || exit 1
done
exit 0
