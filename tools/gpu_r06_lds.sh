# round 6: the quad kernel's LDS tables in place (22.5 KB per workgroup: 4
# workgroups per CU at <= 128 VGPRs; build_variants/lds) against the committed
# build (build_variants/cplx), then the low-rank GPU tests and BPSK / QPSK timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
: > gpurun_out/ab_lds.txt
for t in 9 12 16 20 24; do
  timeout -k 10 150 python -u tools/ab_libs.py build_variants/cplx build_variants/lds --leg lowrank --taps $t --frames 65536 --rounds 7 >> gpurun_out/ab_lds.txt 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cov_quad2_gpu.py tests/test_cov_taps_gpu.py tests/test_cov_lowrank_gpu.py tests/test_cov_mp_gpu.py tests/test_cov_cm_gpu.py tests/test_variants_gpu.py > gpurun_out/lds_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_cplx.py --taps 9 12 16 20 24 > gpurun_out/ab_cplx_lds.txt 2>&1 &&
echo "lds done"
