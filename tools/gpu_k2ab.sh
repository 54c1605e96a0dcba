# K2y split-count A/B with the k2 probe (stage times per binding distribution)
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-k2ab}
mkdir -p $OUT
for s in 8 16 24; do
  echo "splits=$s"; CRANE_K2Y_SPLITS=$s timeout -k 10 120 python tools/k2_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
