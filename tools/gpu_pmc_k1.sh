# Instruction-mix PMC passes for K1 at 4M nodes (tools/stream_bench.py, read flush).
# Usage: bash tools/gpu_pmc_k1.sh <tag>
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmck1_$1
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 $GRAFT_REPO_ROOT/tools/stream_bench.py --k2 auto --reps 2 --flush read"
i=0
for pass in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $OUT -o p$i -- $CMD > $OUT/p$i.log 2>&1
    rc=$?
    echo "pass $i rc=$rc" >> $OUT/status.txt
    case $rc in 0) ;; *) tail -5 $OUT/p$i.log; exit $rc;; esac
done
python3 tools/pmc_agg.py $OUT k1_node_pass k3s_eval
