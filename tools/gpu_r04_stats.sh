# round 4: rocprofv3 kernel-trace statistics of the full bench and of the headline alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/stats.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_head" -o run \
    -- python3 "$R/bench.py" --no-extras --no-cpu-baseline > "$R/gpurun_out/stats_head.log" 2>&1 &&
echo "stats done"
