set -o pipefail
O=gpurun_out/rccl_overhead.txt; : > $O
for a in "none" "nccl" "gloo" "nccl --destroy" "none" "nccl"; do
  timeout -k 10 120 python3 tools/rccl_overhead.py --pg $a >> $O 2>/dev/null || exit $?
done
