# tools/rccl_overhead.py variants in fresh processes (gpurun_out/rccl_overhead.txt)
set -o pipefail
O=gpurun_out/rccl_overhead.txt; : > $O
for a in "none" "nccl" "nccl --barrier" "nccl --bcast" "nccl --bcast --barrier" "none" "nccl --bcast --barrier"; do
  timeout -k 10 120 python3 tools/rccl_overhead.py --pg $a 2>/dev/null | grep pg= >> $O || exit $?
done
