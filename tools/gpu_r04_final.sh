# round 4 close: the GPU gate, the default bench, then the rocprofv3 kernel statistics
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_r04_check.sh && bash tools/gpu_r04_stats.sh
