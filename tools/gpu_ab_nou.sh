# round 5 (timing-only ablation): the headline without the read-out's u load at the wave's end
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/nou"}
timeout -k 10 300 python -u tools/ab_libs.py $V --leg headline --frames 65536 --reps 20 --rounds 9 > gpurun_out/ab_nou.txt 2>&1
