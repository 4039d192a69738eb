# round 5: serialized-load fixes (ref_fc tx_pre in LDS + load order, cm_real branch-free loads), interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/tp build_variants/tpo build_variants/tpo2"}
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fcref --frames 65536 --reps 20 > gpurun_out/ab_lat.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fcref --frames 1048576 --reps 10 >> gpurun_out/ab_lat.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg c5ref_fc --frames 1048576 --reps 5 --rounds 3 >> gpurun_out/ab_lat.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cm --taps 53 --frames 65536 --reps 20 >> gpurun_out/ab_lat.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cm --taps 16 --frames 65536 --reps 20 >> gpurun_out/ab_lat.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py $V --leg cm --taps 53 --frames 1048576 --reps 10 >> gpurun_out/ab_lat.txt 2>&1
