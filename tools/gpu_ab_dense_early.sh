# round 5: dense-C solve with C's 28 block loads and the frame's tx / rx in one round trip, interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/de"}
O=gpurun_out/ab_dense_early.txt
timeout -k 10 200 python -u tools/ab_libs.py $V --leg dense --frames 65536 --reps 20 --rounds 9 > $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg headline --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg dense --frames 1048576 --reps 3 --rounds 5 >> $O 2>&1
