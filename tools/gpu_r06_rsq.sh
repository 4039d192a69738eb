# round 6: A/B of the headline's pivot reciprocal square root on the pivot lane
# (rsq_lane) against the committed build (build_variants/pre), then the GPU gate,
# smoke, the default bench, PMC legs and rocprofv3 kernel statistics of the new build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab_libs.py build_variants/pre 80211parallelestimation_amd --leg headline --frames 65536 --rounds 7 > gpurun_out/ab_rsq_headline.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py build_variants/pre 80211parallelestimation_amd --leg config5 --frames 1048576 --rounds 5 > gpurun_out/ab_rsq_config5.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py --extras-out gpurun_out/bench_extras.json > gpurun_out/bench.out 2> gpurun_out/bench.err &&
timeout -k 10 600 bash tools/pmc_legs.sh headline ref lowrank16 lowrank24 > gpurun_out/pmc_r06.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline --extras-out "$R/gpurun_out/stats_extras.json" > "$R/gpurun_out/stats.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_head" -o run \
    -- python3 "$R/bench.py" --no-extras --no-cpu-baseline --extras-out "$R/gpurun_out/stats_head_extras.json" > "$R/gpurun_out/stats_head.log" 2>&1 &&
echo "r06 rsq done"
