# Run-to-run spread of the default bench line on one box (box variance):
# the headline, the cold legs and the config-3 matrix kernel, N back-to-back runs.
#   bash tools/gpu_variance.sh <tag> [N]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-var}
mkdir -p $OUT
for i in $(seq 1 ${2:-3}); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/run$i.log 2>&1 || { tail -20 $OUT/run$i.log; exit 1; }
  python3 - $OUT/run$i.log $i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rc = d["roofline_cold"]
m3 = d.get("matrix_config3", {})
print(f"run {sys.argv[2]}: value {d['value']:.4g} ms/batch {d['ms_per_step']} kernels {d['kernel_ms']} "
      f"cold k2 {rc['k2']['ms']} k2ts {rc['k2_timestamp_path']['ms']} k1 {rc['k1']['ms']} k1r {rc['k1_records']['ms']} "
      f"matrix3 {m3.get('kernel_ms')} ms dropin {d['dropin'].get('dropin_ms_per_pod')} select {d['select_config3']['adaptive_percentage'].get('ms')}")
PY
done
rocm-smi --showclocks --showpower --showtemp > $OUT/smi.txt 2>&1 || true
