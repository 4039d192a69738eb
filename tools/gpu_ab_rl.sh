set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_sp.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cov_taps_gpu.py tests/test_cov_lowrank_gpu.py -m gpu > gpurun_out/sp_tests.log 2>&1
for T in 53 40 33 24 17; do timeout -k 10 200 python -u tools/ab_libs.py build_variants/sp0 build_variants/sp1 --leg lowrank --taps $T --frames 65536 >> gpurun_out/ab_sp.txt 2>&1 || exit 1; done
