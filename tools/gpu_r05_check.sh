# round 5: new/changed GPU tests first, then the whole GPU gate, then the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
T="${TESTS:-tests/test_headline_batch_gpu.py tests/test_cov_cm_gpu.py tests/test_variants_gpu.py}"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T -m gpu > gpurun_out/gpu_new.log 2>&1 &&
if [ -n "$FULL" ]; then timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1; fi &&
if [ -n "$BENCH" ]; then timeout -k 10 600 python -u bench.py --extras-out gpurun_out/bench_extras.json > gpurun_out/bench.out 2> gpurun_out/bench.err; fi
