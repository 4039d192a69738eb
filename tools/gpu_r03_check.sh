# round 3: the whole GPU gate, then the headline bench alone (perf sanity)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err
