# round 4: Toeplitz lane / quad kernels -- the low-rank gates, then the low-rank timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_cov_taps_gpu.py tests/test_cov_lowrank_gpu.py tests/test_cov_cm_gpu.py tests/test_bigindex_gpu.py tests/test_variants_gpu.py -m gpu > gpurun_out/taps_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/quick_lowrank.py 20 > gpurun_out/quick_lowrank.json 2> gpurun_out/quick_lowrank.err
