# round 5: the tap-domain wave kernel (mmse_lr_kernel<0, true>, 53 taps) variants, interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/keep"}
timeout -k 10 300 python -u tools/ab_libs.py $V --leg lowrank --taps 53 --frames 65536 --reps 20 --rounds 7 > gpurun_out/ab_taps.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg lowrank --taps 40 --frames 65536 --reps 20 --rounds 5 >> gpurun_out/ab_taps.txt 2>&1
