# round 5: mmse_ref_flat_kernel with / without the next chunk's pilots prefetched
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V="build_variants/ref0 build_variants/ref1"
timeout -k 10 300 python -u tools/ab_libs.py $V --leg refmm --frames 1048576 --reps 20 > gpurun_out/ab_ref.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg refmm --frames 65536 --reps 50 >> gpurun_out/ab_ref.txt 2>&1
