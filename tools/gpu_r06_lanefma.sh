# round 6: the lane kernels' complex-symbol correction as FMA chains
# (build_variants/fma) against the committed build (build_variants/head):
# BPSK / QPSK timing per build (twice, interleaved), then the low-rank GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
: > gpurun_out/ab_lanefma.txt
for r in 1 2; do
  for b in head fma; do
    echo "## $b (round $r)" >> gpurun_out/ab_lanefma.txt
    timeout -k 10 150 python -u tools/ab_cplx.py --taps 2 4 8 --lib build_variants/$b/libwce.so >> gpurun_out/ab_lanefma.txt 2>&1 || exit $?
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cov_lowrank_gpu.py tests/test_cov_taps_gpu.py tests/test_cov_mp_gpu.py tests/test_cov_cm_gpu.py > gpurun_out/lanefma_tests.log 2>&1 &&
echo "lanefma done"
