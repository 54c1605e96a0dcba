# K2 large form: prefetch copied at the loop top (k2c, the tree's library) vs sra, with the
# option combinations (workgroup size, region size, count/offset layout); hot-value tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hot" > $O/pytest_hot.log 2>&1 || { tail -30 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
for rep in 1 2; do for v in sra k2c; do
  cp crane-scheduler_amd/lib_ab/lib_$v.so $L
  for o in k2l_threads=512 k2l_threads=1024 "k2l_region=2048 --opt k2l_co_t=1" "k2l_threads=1024 --opt k2l_co_t=1"; do
    timeout -k 10 300 python -u bench.py --leg cold --steps 5 --opt $o > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/cold.log').read().strip().splitlines()[-1]); print('$v', '$o', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'])"
  done
done; done
