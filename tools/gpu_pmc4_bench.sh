# Config-4 PMC summary, then the config-3 and config-4 bench lines with the PMC traffic attached.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
H=$(python3 -c "import bench; print(bench.src_hash())")
bash tools/gpu_pmc.sh h2 4 || exit 1
cp gpurun_out/pmc_h2_4/summary.json profiles/pmc/config4_$H.json
mkdir -p gpurun_out/b34
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --no-greedy > gpurun_out/b34/bench4.log 2>&1 || { tail gpurun_out/b34/bench4.log; exit 1; }
timeout -k 10 300 python bench.py --no-greedy --no-extras > gpurun_out/b34/bench3.log 2>&1 || { tail gpurun_out/b34/bench3.log; exit 1; }
tail -1 gpurun_out/b34/bench4.log | cut -c1-400
