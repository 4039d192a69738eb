# round 6: the GPU gate, the launcher-less two-rank rehearsal
# (bench.py --gpus 2 starts its own ranks; gloo, both on GPU 0) and the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
WCE_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
    --extras-out gpurun_out/bench_2rank_launcher_extras.json > gpurun_out/bench_2rank_launcher.json 2> gpurun_out/bench_2rank_launcher.err &&
timeout -k 10 600 python -u bench.py --extras-out gpurun_out/bench_extras.json > gpurun_out/bench.out 2> gpurun_out/bench.err &&
echo "r06 check done"
