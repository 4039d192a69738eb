# round 6: the rank 9..16 quad kernel with fused-DPP Cholesky updates: the low-rank
# tests, then an A/B at 16 taps (default | separate movs | wave kernel) and ranks 17..32
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cov_lowrank_gpu.py tests/test_cov_taps_gpu.py tests/test_cov_cm_gpu.py tests/test_cov_quad2_gpu.py tests/test_isa.py -m "gpu or not gpu" > gpurun_out/quad_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_lowrank.py --taps 16 12 24 > gpurun_out/ab_lowrank_quad.txt 2>&1 &&
echo "r06 quad done"
