set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_store8.txt
for F in 1048576 65536; do for T in 8 4 2; do timeout -k 10 200 python -u tools/ab_libs.py build_variants/s4 build_variants/s8 --leg lowrank --taps $T --frames $F >> gpurun_out/ab_store8.txt 2>&1 || exit 1; done; done
