# round 6, final: the whole GPU gate, smoke, the default bench (its traffic from
# profiles/r06_pmc_legs.json, every leg refreshed by tools/pmc_legs.sh), the PMC leg of
# the quad kernel changed since (lowrank16) and the
# rocprofv3 kernel statistics of the full bench and of the headline alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py --extras-out gpurun_out/bench_extras.json > gpurun_out/bench.out 2> gpurun_out/bench.err &&
timeout -k 10 200 bash tools/pmc_legs.sh lowrank16 > gpurun_out/pmc_r06.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --extras-out "$R/gpurun_out/stats_extras.json" > "$R/gpurun_out/stats.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_head" -o run \
    -- python3 "$R/bench.py" --no-extras --no-cpu-baseline --extras-out "$R/gpurun_out/stats_head_extras.json" > "$R/gpurun_out/stats_head.log" 2>&1 &&
echo "r06 final2 done"
