# Round 4, first GPU pass of the incremental drop-in: the new GPU tests, then the drop-in leg
# at config 2 (5k nodes) and config 3 (100k nodes).   bash tools/gpu_r04a.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
timeout -k 10 300 python -u tools/dropin_probe.py 5000 256 > $OUT/dropin_5k.json 2> $OUT/dropin_5k.err || { tail -30 $OUT/dropin_5k.err; exit 1; }
timeout -k 10 400 python -u tools/dropin_probe.py 100000 256 > $OUT/dropin_100k.json 2> $OUT/dropin_100k.err || { tail -30 $OUT/dropin_100k.err; exit 1; }
cut -c1-2500 $OUT/dropin_5k.json; echo; cut -c1-3500 $OUT/dropin_100k.json
# cold 4M-node K1 / K2 legs: the fused node pass and the split forms
bash tools/gpu_r04c.sh ${1:-r04a} "default;k1_threads=128;k1_split=1;k1_split=1 emit_threads=64;k1_split=1 emit_threads=64 k1_count_form=1;k1_split=1 emit_threads=64 k1_count_form=2;k1_split=1 emit_threads=64 k1_count_form=3" || exit 1
