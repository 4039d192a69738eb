# round 5: apply_kernel with a per-tile keep mask (one skip[] load per lane per tile), A/B + the skip-path tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/keep"}
O=gpurun_out/ab_keep.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cov_cm_gpu.py tests/test_parity_gpu.py -m gpu > gpurun_out/keep_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg apply --frames 65536 --reps 20 --rounds 7 > $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg apply --frames 1048576 --reps 10 >> $O 2>&1
