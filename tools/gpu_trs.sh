cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/trs
timeout -k 10 200 python -u tools/trace_step.py --config 3 --nodes 4000000 --bindings 16000000 --reps 3 --opt k1_stream=1 > gpurun_out/trs/t.json 2>gpurun_out/trs/t.err || { tail gpurun_out/trs/t.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/trs/t.json')); k=d['K1']; print(k['span'], k['phases'], k.get('sub'))"
