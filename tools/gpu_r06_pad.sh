# round 6: A/B of the quad / quad2 kernels' LDS tables at odd 16-B-slot row
# pitches (build_variants/pad) against the committed build (build_variants/rsq),
# then the low-rank GPU tests on the padded build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
: > gpurun_out/ab_pad.txt
for t in 12 16 20 24 32; do
  timeout -k 10 120 python -u tools/ab_libs.py build_variants/rsq build_variants/pad --leg lowrank --taps $t --frames 65536 --rounds 5 >> gpurun_out/ab_pad.txt 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cov_quad2_gpu.py tests/test_cov_taps_gpu.py tests/test_cov_lowrank_gpu.py tests/test_cov_mp_gpu.py > gpurun_out/pad_tests.log 2>&1 &&
timeout -k 10 120 bash tools/pmc_legs.sh lowrank16 lowrank24 > gpurun_out/pmc_pad.log 2>&1 &&
echo "pad done"
