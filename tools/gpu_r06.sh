# Round-6 GPU runs on the current tree (one gpurun call per stage):
#   bash tools/gpu_r06.sh <tag> quick [pytest files...]  the named GPU test files + a 20-step bench line
#   bash tools/gpu_r06.sh <tag> verify   GPU suite, smoke, the driver's bench command
#   bash tools/gpu_r06.sh <tag> bench    default bench line + the 20-step driver command + one-batch rocprof
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r06}
O=gpurun_out/$T
mkdir -p $O
H=$(python3 -c "import bench; print(bench.src_hash())")
echo "src_hash $H"
export TMPDIR=/tmp
ST=$2
shift 2
case $ST in
quick)
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -80 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $O/bench20.log 2>&1 || { tail -30 $O/bench20.log; exit 1; }
  tail -1 $O/bench20.log | cut -c1-3000
  ;;
verify)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -80 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -30 $O/bench20.log; exit 1; }
  tail -1 $O/bench20.log | cut -c1-1500
  ;;
bench)
  timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-600
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -30 $O/bench20.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof1 -o bench1 \
      -- python3 $GRAFT_REPO_ROOT/bench.py --inflight 1 --no-cpu-baseline --no-greedy --no-extras > $O/prof1.log 2>&1 || { tail -20 $O/prof1.log; exit 1; }
  python3 tools/kstats.py $O/prof1/bench1_kernel_stats.csv
  ;;
*) echo "stage: quick | verify | bench"; exit 2;;
esac
echo "src_hash $H"
