# GPU: parity tests then the K3 A/B sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 600 python tools/k3_ab.py > gpurun_out/k3_ab.json 2> gpurun_out/k3_ab.err
