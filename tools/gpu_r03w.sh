# selection walk with the in-range nodes' A ranks kept in the list (sra) vs g4: selection tests on
# sra, the config-3 queue timed per library; then the cold K2 large-form option sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash tools/gpu_select_ab.sh r03w g4 sra || exit 1
timeout -k 10 600 bash tools/gpu_r03v.sh || exit 1
