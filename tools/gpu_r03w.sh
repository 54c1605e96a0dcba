# selection walk: in-range nodes' A ranks kept in the list (sra), + the select word folded into the
# rank round trip (sr2, the tree's library) vs g4: selection tests on sr2, the config-3 queue timed
# per library; the drop-in leg with the branch-free feasible list; the cold K2 option sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash tools/gpu_select_ab.sh r03w g4 sra sr2 || exit 1
timeout -k 10 600 python tools/dropin_probe.py > gpurun_out/r03w/dropin.json 2> gpurun_out/r03w/dropin.err || { tail gpurun_out/r03w/dropin.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03w/dropin.json')); d.pop('workload'); d.get('cpu_same_harness',{}).pop('how',None); print(json.dumps(d)[:1200])"
timeout -k 10 600 bash tools/gpu_r03v.sh || exit 1
