# round 6: the quad kernels' complex-symbol correction in the tap domain -- the
# low-rank GPU tests (QPSK / 16-QAM cases included), then BPSK vs QPSK timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cov_quad2_gpu.py tests/test_cov_taps_gpu.py tests/test_cov_lowrank_gpu.py tests/test_cov_mp_gpu.py tests/test_cov_cm_gpu.py tests/test_variants_gpu.py tests/test_accuracy_gpu.py > gpurun_out/cplx_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_cplx.py --taps 12 16 20 24 > gpurun_out/ab_cplx_new.txt 2>&1 &&
echo "cplx done"
