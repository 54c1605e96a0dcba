# config 3: K1 workgroups of 128 nodes (782 workgroups, half the epilogue each) vs 256, one batch
# (kernel times) and 4 in flight
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03z; mkdir -p $O
for rep in 1 2; do for o in k1_threads=256 k1_threads=128; do
  timeout -k 10 200 python tools/inflight_probe.py --inflight 1,4 --bound --opt $o > $O/inf_$o.json 2>&1 || { tail $O/inf_$o.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/inf_$o.json').read().strip().splitlines()[-1]); print('$o 1/4', d['inflight1']['ms_per_step'], d['inflight4']['ms_per_step'], d['inflight4']['keys_equal'])"
  timeout -k 10 200 python tools/trace_step.py --config 3 --opt $o > $O/t3_$o.json 2> $O/t3_$o.err || { tail $O/t3_$o.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/t3_$o.json'))
print('$o', {k: (d[k]['span'], d[k]['workgroups']) for k in ('K2x','K1','K3s') if k in d})"
done; done
# the collective path rehearsed on one rank: all-reduce on its own stream vs on an engine stream
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --config 3 --steps 512 --no-extras --no-cpu-baseline --no-greedy > $O/b3.log 2>&1 || { tail -30 $O/b3.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b3.log').read().strip().splitlines()[-1]); print('no collective', d['ms_per_step'])"
for s in own engine; do for g in 64 128; do
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2954$((g % 10)) timeout -k 10 300 python -u bench.py --config 3 --steps 512 --rehearse-collective --ar-stream $s --ar-group $g --no-extras --no-cpu-baseline --no-greedy > $O/r3.log 2>&1 || { tail -30 $O/r3.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/r3.log').read().strip().splitlines()[-1]); print('rehearse $s G=$g', d['ms_per_step'], d['allreduce_ms'], d['keys_match_1gpu'])"
done; done
done
