# round 4: tap-domain Gram (pair DFTs) -- its tests, then ablation A/B and the low-rank timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_cov_taps_gpu.py tests/test_cov_cm_gpu.py -m gpu > gpurun_out/taps_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py build_variants/base build_variants/nodft build_variants/noout build_variants/w2 --leg lowrank --taps 53 --frames 65536 > gpurun_out/ab_taps.txt 2>&1 &&
timeout -k 10 300 python -u tools/quick_lowrank.py 20 > gpurun_out/quick_lowrank.json 2> gpurun_out/quick_lowrank.err
