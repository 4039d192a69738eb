# round 5: the tap-domain wave kernel at K0 >= 1 with E, the tap map and s_j in the frame's round trip, interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/early"}
O=gpurun_out/ab_taps2.txt
timeout -k 10 200 python -u tools/ab_libs.py $V --leg lowrank --taps 24 --frames 65536 --reps 20 --rounds 7 > $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg lowrank --taps 32 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg lowrank --taps 40 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg lowrank --taps 53 --frames 65536 --reps 20 --rounds 5 >> $O 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cov_taps_gpu.py tests/test_cov_lowrank_gpu.py -m gpu > gpurun_out/taps2_tests.log 2>&1
