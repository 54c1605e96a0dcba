set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/stream_bench.py --k1-threads 128 > gpurun_out/stream.json 2>gpurun_out/stream.err || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
