set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_fpw.txt
for T in 4 8 6; do timeout -k 10 200 python -u tools/ab_libs.py build_variants/f64 build_variants/f32 build_variants/f16 --leg lowrank --taps $T --frames 65536 >> gpurun_out/ab_fpw.txt 2>&1 || exit 1; done
