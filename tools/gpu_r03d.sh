# full GPU suite + cold leg + config-3/4 headline (no extras)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --leg cold --steps 5 > $O/cold.log 2>&1 || { tail -30 $O/cold.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/cold.log').read().strip().splitlines()[-1]); print('cold', d['k2']['ms'], d['k2']['frac'], d['k2']['kernels'], d['k1']['ms'], d['k1']['frac'])"
for c in 3 4; do
timeout -k 10 300 python -u bench.py --config $c --steps 50 --no-extras --no-cpu-baseline --no-greedy > $O/b$c.log 2>&1 || { tail -30 $O/b$c.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b$c.log').read().strip().splitlines()[-1]); print('config$c', d['ms_per_step'], d['batches_in_flight']['batch_latency_ms'], d['kernel_ms'])"
done
