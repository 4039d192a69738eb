# round 5: cm_cplx_kernel (QPSK constant-modulus frames) with branch-free tile loads, interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/cmc"}
O=gpurun_out/ab_cmq.txt
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cmq --taps 53 --frames 65536 --reps 20 --rounds 7 > $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cmq --taps 16 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cmq --taps 53 --frames 524288 --reps 10 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cm --taps 53 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1
