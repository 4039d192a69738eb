# round 6: REF read-out, one frame per wave (which 0 = 4) against one element per thread (3);
# the quad kernel's pair-form Gram / read-out: the low-rank tests and a timing at 12 / 16 taps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_variants_gpu.py tests/test_cov_lowrank_gpu.py tests/test_cov_taps_gpu.py tests/test_cov_cm_gpu.py tests/test_cov_quad2_gpu.py tests/test_bigindex_gpu.py -m gpu > gpurun_out/refw_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 3 4 1 --frames 1048576 --rounds 5 > gpurun_out/ab_refw_1m.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 3 4 1 --frames 262144 --rounds 5 > gpurun_out/ab_refw_256k.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_lowrank.py --taps 16 12 10 > gpurun_out/ab_lowrank_quad_pairs.txt 2>&1 &&
echo "r06 refw done"
