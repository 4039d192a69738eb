# round 5: ref_fc_kernel variants (tools/variants.sh builds under build_variants/), interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/C build_variants/F build_variants/G build_variants/H"}
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fcref --frames 65536 --reps 20 > gpurun_out/ab_fc.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fcref --frames 1048576 --reps 10 >> gpurun_out/ab_fc.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg c5ref_fc --frames 1048576 --reps 5 --rounds 3 >> gpurun_out/ab_fc.txt 2>&1
