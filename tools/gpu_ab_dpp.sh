set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_dpp.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/dpp_tests.log 2>&1
for L in "dense" "r1dense" "config5" "headline"; do timeout -k 10 200 python -u tools/ab_libs.py build_variants/dprev build_variants/dmov --leg $L >> gpurun_out/ab_dpp.txt 2>&1 || exit 1; done
for T in 53 24 17; do timeout -k 10 200 python -u tools/ab_libs.py build_variants/dprev build_variants/dmov --leg lowrank --taps $T --frames 65536 >> gpurun_out/ab_dpp.txt 2>&1 || exit 1; done
