# round 5: H = C W below 131,072 frames: matvec_kernel (one tile per wave) vs the streaming apply_kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V="build_variants/ap4 build_variants/ap1 build_variants/ap0"
: > gpurun_out/ab_apply.txt
for n in 16384 65536 131072; do
  timeout -k 10 200 python -u tools/ab_libs.py $V --leg apply --frames $n --reps 20 >> gpurun_out/ab_apply.txt 2>&1 || exit $?
done
