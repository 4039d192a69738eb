#!/bin/bash
# HBM traffic of the configs[1] LS kernel alone: tools/ab_ls.py (1,048,576
# frames, every dispatch the same size) under rocprofv3 --pmc, one pass per
# counter group -> gpurun_out/pmc_ls/<pass>/, summarised per dispatch.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_ls
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run --pmc "$@" \
     -- python3 "$ROOT/tools/ab_ls.py" "$ROOT/80211parallelestimation_amd" --rounds 1 --reps 3 > "$OUT/$name.log" 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
python3 "$ROOT/tools/pmc_summary.py" "$OUT" "$ROOT/gpurun_out/pmc_ls.json" > /dev/null && echo "pmc_ls done"
