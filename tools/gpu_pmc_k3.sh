# rocprofv3 PMC passes over the K3 sweep driver (one counter group per pass,
# --pmc only, no trace domains).  Usage: bash tools/gpu_pmc_k3.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-k3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
CMD="python3 $GRAFT_REPO_ROOT/tools/k3_sweep.py"
run() {  # name counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o $name -- $CMD > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc" >> $OUT/status.txt
    case $rc in 124|134|137|139) exit $rc;; esac
    return 0
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VALU
run sq2 SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
run l2 TCC_HIT_sum TCC_MISS_sum
run lds SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM
exit 0
