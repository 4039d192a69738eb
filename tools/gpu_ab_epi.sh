# round 5: the fused configs[4] epilogue (mmse_solve_ls_kernel) with every load issued before the first use, interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/epi"}
O=gpurun_out/ab_epi.txt
timeout -k 10 300 python -u tools/ab_libs.py $V --leg config5 --frames 262144 --reps 5 --rounds 7 > $O 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg config5 --frames 1048576 --reps 3 --rounds 5 >> $O 2>&1
