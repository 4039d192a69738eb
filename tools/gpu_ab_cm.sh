set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_cm.txt
for F in 65536 1048576; do for T in 53 16; do timeout -k 10 200 python -u tools/ab_libs.py build_variants/cmK build_variants/cmS --leg cm --taps $T --frames $F >> gpurun_out/ab_cm.txt 2>&1 || exit 1; done; done
