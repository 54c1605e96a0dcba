# g4 (the tree's library) vs base A/B (cold 4M K1, config-3 in flight), then the round-end
# verification on the tree: GPU suite, smoke, bench line, cold stream, rocprof stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash tools/gpu_r03t.sh || exit 1
bash tools/gpu_verify.sh r03_v2 || exit 1
