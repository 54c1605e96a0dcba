# Round-end evidence on the current tree: GPU suite + smoke + bench + stream + rocprof stats
# (tools/gpu_verify.sh), PMC summaries of configs 3, 2, 3m, 4m, 4 for these kernel sources
# (tools/gpu_pmc.sh), then the config-3 and config-4 bench lines with that traffic attached.
#   bash tools/gpu_final.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1
H=$(python3 -c "import bench; print(bench.src_hash())")
bash tools/gpu_verify.sh $T || exit 1
bash tools/gpu_pmc.sh $T "3 2 3m 4m 4" || exit 1
for c in 3 2 3m 4m 4; do cp gpurun_out/pmc_${T}_$c/summary.json profiles/pmc/config${c}_$H.json; done
mkdir -p gpurun_out/$T/pmc_json && cp profiles/pmc/config*_$H.json gpurun_out/$T/pmc_json/
timeout -k 10 300 python bench.py > gpurun_out/$T/bench_traffic.log 2>&1 || { tail gpurun_out/$T/bench_traffic.log; exit 1; }
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/$T/bench4_traffic.log 2>&1 || { tail gpurun_out/$T/bench4_traffic.log; exit 1; }
echo "hash $H"
