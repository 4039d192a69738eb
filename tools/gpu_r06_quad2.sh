# round 6: ranks 17..32 on mmse_lr_quad2_kernel -- its tests and the tests that
# name the rank-24 kernel, the ISA-independent variant gate, then an A/B against
# the wave kernel (and, at rank 24, the fused-DPP Cholesky against separate movs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cov_quad2_gpu.py tests/test_cov_taps_gpu.py tests/test_cov_cm_gpu.py tests/test_bigindex_gpu.py tests/test_variants_gpu.py tests/test_cov_lowrank_gpu.py tests/test_parity_gpu.py tests/test_chunks_gpu.py -m gpu > gpurun_out/quad2_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_lowrank.py > gpurun_out/ab_lowrank.txt 2>&1 &&
echo "r06 quad2 done"
