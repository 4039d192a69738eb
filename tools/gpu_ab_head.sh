# round 5: the headline kernel family with the rank-1 factors loaded in the frame's round trip, interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/early"}
timeout -k 10 300 python -u tools/ab_libs.py $V --leg headline --frames 65536 --reps 20 --rounds 9 > gpurun_out/ab_head.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg config5 --frames 262144 --reps 5 --rounds 5 >> gpurun_out/ab_head.txt 2>&1
