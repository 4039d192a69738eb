# round 5: LDS staging with every load issued before the first store (one round trip per workgroup), interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=${V:-"build_variants/base build_variants/stage"}
O=gpurun_out/ab_stage.txt
timeout -k 10 200 python -u tools/ab_libs.py $V --leg apply --frames 65536 --reps 20 --rounds 7 > $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg apply --frames 1048576 --reps 10 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fcref --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg fcref --frames 1048576 --reps 10 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cm --taps 53 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg cm --taps 16 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg lowrank --taps 4 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg lowrank --taps 8 --frames 65536 --reps 20 --rounds 7 >> $O 2>&1 &&
timeout -k 10 200 python -u tools/ab_libs.py $V --leg lowrank --taps 8 --frames 1048576 --reps 10 >> $O 2>&1
