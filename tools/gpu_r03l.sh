set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 600 python tools/dropin_probe.py > $O/dropin.json 2> $O/dropin.err || { tail $O/dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin.json')); d.pop('workload'); d['cpu_same_harness'].pop('how'); print(json.dumps(d))"
for g in 32 64 128; do
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$((g % 10)) timeout -k 10 300 python -u bench.py --config 3 --steps 256 --rehearse-collective --ar-group $g --no-extras --no-cpu-baseline --no-greedy > $O/r3.log 2>&1 || { tail -30 $O/r3.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/r3.log').read().strip().splitlines()[-1]); print('rehearse3 G=$g', d['ms_per_step'], d['allreduce_ms'], d['keys_match_1gpu'])"
done
timeout -k 10 300 python -u bench.py --config 3 --steps 256 --no-extras --no-cpu-baseline --no-greedy > $O/b3.log 2>&1 || { tail -30 $O/b3.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b3.log').read().strip().splitlines()[-1]); print('config3', d['ms_per_step'], d['batches_in_flight']['batch_latency_ms'], d['kernel_ms'])"
