# round 6: REF read-out, one frame per wave (which 0 = 4) against one element per thread (3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_variants_gpu.py -m gpu > gpurun_out/refw_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 3 4 1 --frames 1048576 --rounds 5 > gpurun_out/ab_refw_1m.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 3 4 1 --frames 262144 --rounds 5 > gpurun_out/ab_refw_256k.txt 2>&1 &&
echo "r06 refw done"
