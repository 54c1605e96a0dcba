# GPU: selected parity tests + bench.  Usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-greedy > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
