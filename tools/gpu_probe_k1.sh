# K1 cold-cache ceilings (tools/k1_ceiling.hip) and the SQ instruction counters rocprofv3 offers.
# Usage: bash tools/gpu_probe_k1.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 120 ./tools/bin/k1_ceiling > $OUT/k1_ceiling.json 2>&1 || { cat $OUT/k1_ceiling.json; exit 1; }
cat $OUT/k1_ceiling.json
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $OUT/counters.txt | sort -u > $OUT/sq_counters.txt || true
