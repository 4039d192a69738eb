# round 4: the whole GPU gate, an A/B of library builds, then the full default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
if [ -n "$AB" ]; then timeout -k 10 300 python -u tools/ab_libs.py $AB > gpurun_out/ab.txt 2>&1; fi &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
