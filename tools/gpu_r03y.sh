# large-form K2 with narrower bins (kh: option k2l_hist_kb, Y's LDS histogram per bin) on the cold leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03y; mkdir -p $O
L=crane-scheduler_amd/lib/libcrane_dyn.so
cp $L $O/orig.so
trap 'cp $O/orig.so $L' EXIT
cp crane-scheduler_amd/lib_ab/lib_kh.so $L
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "large_form" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for kb in 128 64 32; do
  timeout -k 10 300 python -u bench.py --leg cold --steps 5 --opt k2l_hist_kb=$kb > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/cold.log').read().strip().splitlines()[-1]); print('hist_kb $kb', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'])"
done; done
# config-4 shard (125k nodes, one round of producers): middle pieces cut (step_pieces 1) vs the
# default gate (off there) and never, one batch and 4 in flight
cp $O/orig.so $L
for o in step_pieces=0 step_pieces=1 step_pieces=2; do
  timeout -k 10 200 python tools/inflight_probe.py --config 4 --inflight 1,4 --bound --opt $o > $O/inf4_$o.json 2>&1 || { tail $O/inf4_$o.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/inf4_$o.json').read().strip().splitlines()[-1]); print('shard $o 1/4', d['inflight1']['ms_per_step'], d['inflight4']['ms_per_step'], d['inflight4']['keys_equal'])"
done
