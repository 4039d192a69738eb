#!/bin/bash
# One gpurun call that regenerates the profiles/ artefacts of a round:
#   1. PMC passes over every bench leg's kernel alone at the bench's launch
#      size (tools/pmc_legs.sh -> pmc_legs.json, read by bench.py)
#   2. the full bench line
#   3. rocprofv3 --kernel-trace --stats of the same bench, and of the
#      headline alone (kernel durations)
# Results land in gpurun_out/; tools/collect_profiles.sh copies them into
# profiles/ under the round prefix.  ROUND=r02 by default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
RND=${ROUND:-r02}
mkdir -p "$R/gpurun_out"
# SKIP_PMC=1: keep the committed PMC legs (valid while the kernels are unchanged)
if [ -z "$SKIP_PMC" ]; then
  cd "$R" && bash tools/pmc_legs.sh > "$R/gpurun_out/pmc_legs.log" 2>&1 || exit $?
  cp "$R/gpurun_out/pmc_legs.json" "$R/profiles/${RND}_pmc_legs.json"   # the bench reads the newest
fi
timeout -k 10 400 python3 "$R/bench.py" > "$R/gpurun_out/bench_full.json" 2> "$R/gpurun_out/bench_full.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/stats.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_head" -o run \
    -- python3 "$R/bench.py" --no-extras --no-cpu-baseline > "$R/gpurun_out/stats_head.log" 2>&1 || exit $?
echo "refresh done"
