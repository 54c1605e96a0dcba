# Step-path probe on the GPU box: step/shard parity tests, phase traces (configs 3 and 4
# shard), bench configs 3 and 4 without the extra legs.   Usage: bash tools/step_probe.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
timeout -k 10 120 python tools/trace_step.py --config 3 > $OUT/trace3.json || exit 1
timeout -k 10 120 python tools/trace_step.py --config 4 > $OUT/trace4.json || exit 1
timeout -k 10 300 python bench.py --config 3 --no-extras --no-cpu-baseline > $OUT/b3.log 2>&1 || { tail -5 $OUT/b3.log; exit 1; }
timeout -k 10 300 python bench.py --config 4 --no-extras > $OUT/b4.log 2>&1 || { tail -5 $OUT/b4.log; exit 1; }
tail -1 $OUT/pytest.log
