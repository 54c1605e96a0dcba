# PMC passes over the cold leg (large-form K2 + K1 at 4M x 16M)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_pmc.sh r03f cold || exit 1
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/pmc_r03f_cold/summary.json"))
for k,v in d["kernels"].items():
    if "crane" in k: print(k, json.dumps({a:round(b,1) for a,b in v.items()}))
PY
