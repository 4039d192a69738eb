set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cov_cm_gpu.py -m gpu > gpurun_out/cm_tests.log 2>&1 &&
V="build_variants/cmO build_variants/cmP build_variants/cmP21 build_variants/cmP11 build_variants/cmP12"
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cm --taps 53 --frames 65536 --reps 20 > gpurun_out/ab_cm.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cm --taps 16 --frames 65536 --reps 20 >> gpurun_out/ab_cm.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg cm --taps 53 --frames 1048576 --reps 10 >> gpurun_out/ab_cm.txt 2>&1
