# Instruction mix of the cold 4M-node K1 forms: rocprofv3 --pmc passes (counters only, one group
# per pass) over bench.py's cold leg, k1_stream 1 and 0; summaries by tools/pmc_summary.py.
# Usage: bash tools/gpu_k1_pmc.sh <tag>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-k1pmc}
for f in ${2:-1 0}; do
    OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_$f
    mkdir -p $OUT
    for pass in "valu SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" "lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES"; do
        set -- $pass
        name=$1; shift
        timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o $name -- python3 $GRAFT_REPO_ROOT/bench.py --leg cold --steps 2 --opt k1_stream=$f > $OUT/$name.log 2>&1
        rc=$?
        echo "$f $name rc=$rc"
        case $rc in 0) ;; *) exit $rc;; esac
    done
    python3 tools/pmc_summary.py $OUT --config cold > $OUT/summary.json || exit 1
    python3 - $OUT/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if "k1" not in k: continue
    w = v.get("SQ_WAVES", 1) or 1
    print(k[:50], {c: round(v[c] / w, 1) for c in sorted(v) if c.startswith("SQ_") and c != "SQ_WAVES"}, "ns", v["_dispatch_ns"])
PY
done
