# round 6: the whole GPU gate, smoke, and the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py --extras-out gpurun_out/bench_extras.json > gpurun_out/bench.out 2> gpurun_out/bench.err &&
echo "r06 full done"
