set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_quad.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cov_lowrank_gpu.py tests/test_cov_taps_gpu.py -m gpu -k "quad or scattered or taps or bigindex" > gpurun_out/taps_tests.log 2>&1
for T in 16 12 9; do timeout -k 10 200 python -u tools/ab_libs.py build_variants/qprev build_variants/qmov --leg lowrank --taps $T --frames 65536 >> gpurun_out/ab_quad.txt 2>&1 || exit 1; done
