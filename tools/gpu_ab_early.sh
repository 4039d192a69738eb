# round 5: rank-1 factor loads in the frame's first round trip, on the per-frame-covariance (TEXTBOOK) leg too
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/early"}
O=gpurun_out/ab_early.txt
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fctb --frames 65536 --reps 20 --rounds 9 > $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg headline --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg fctb --frames 1048576 --reps 5 --rounds 5 >> $O 2>&1
