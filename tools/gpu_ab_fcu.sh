# round 5: TEXTBOOK FRAME_COV factors (LT_LS + u = Mu h) in one launch, tests + interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/fcu"}
O=gpurun_out/ab_fcu.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_framecov_gpu.py tests/test_matlab_gpu.py -m gpu > gpurun_out/fcu_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fctb --frames 65536 --reps 20 --rounds 9 > $O 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg fctb --frames 1048576 --reps 5 --rounds 5 >> $O 2>&1
