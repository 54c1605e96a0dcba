# Selection tests on the current build, then the selection leg timed with engine builds
# crane-scheduler_amd/lib_ab/lib_<V>.so swapped in.   Usage: bash tools/gpu_select_ab.sh <tag> V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
timeout -k 10 300 python -u -m pytest tests/test_select.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp $L $O/orig.so
for v in "$@"; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L || { cp $O/orig.so $L; exit 1; }
  timeout -k 10 300 python tools/select_probe.py > $O/sel_$v.json 2>&1 || { tail $O/sel_$v.json; cp $O/orig.so $L; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/sel_$v.json').read().strip().splitlines()[-1]); print('$v', d['adaptive_percentage']['ms'], d['adaptive_percentage']['kernel_ms'], d['percentage_100']['ms'])"
done
cp $O/orig.so $L
