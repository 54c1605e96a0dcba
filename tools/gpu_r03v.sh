# cold 4M K2 large-form options (region size, workgroup size, count/offset layout), twice each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03v; mkdir -p $O
for rep in 1 2; do
for o in k2l_region=4096 k2l_region=2048 k2l_threads=1024 k2l_co_t=1; do
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 --opt $o > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold.log').read().strip().splitlines()[-1]); print('$o', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'], d['k1']['ms'], d['k1']['frac'], d['k1_records']['ms'], d['k1_records']['frac'])"
done
done
