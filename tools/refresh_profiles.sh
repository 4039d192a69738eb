#!/bin/bash
# One gpurun call that regenerates every profiles/ artefact of a round:
#   1. PMC passes over the headline alone (-> pmc_headline.json: per-frame
#      counters of the headline kernel, undiluted by other modes' launches of
#      the same kernel) and over all bench legs (-> pmc_summary.json)
#   2. the full bench line (reads the fresh PMC summary for "traffic")
#   3. rocprofv3 --kernel-trace --stats of the same bench (kernel durations)
# Results land in gpurun_out/; copy them into profiles/ with the round prefix
# (tools/collect_profiles.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R" && PMC_DIR=pmc_head bash tools/pmc_passes.sh > "$R/gpurun_out/pmc_head_passes.log" 2>&1 || exit $?
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_head" "$R/gpurun_out/pmc_headline.json" > /dev/null || exit $?
cd "$R" && PMC_EXTRAS=1 bash tools/pmc_passes.sh > "$R/gpurun_out/pmc_passes.log" 2>&1 || exit $?
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc" "$R/gpurun_out/pmc_summary.json" > /dev/null || exit $?
cd "$R" && bash tools/pmc_ls.sh > "$R/gpurun_out/pmc_ls_passes.log" 2>&1 || exit $?
RND=${ROUND:-r01}   # the bench reads the newest profiles/*_pmc_*.json: overwrite this round's
cp "$R/gpurun_out/pmc_ls.json" "$R/profiles/${RND}_pmc_ls.json"
cp "$R/gpurun_out/pmc_summary.json" "$R/profiles/${RND}_pmc_summary.json"
cp "$R/gpurun_out/pmc_headline.json" "$R/profiles/${RND}_pmc_headline.json"
timeout -k 10 400 python3 "$R/bench.py" > "$R/gpurun_out/bench_full.json" 2> "$R/gpurun_out/bench_full.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/stats.log" 2>&1 || exit $?
# headline only: the per-launch average of the headline kernel, undiluted by
# the other modes' launches of the same kernel (REF mode, FRAME_COV)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_head" -o run \
    -- python3 "$R/bench.py" --no-extras --no-cpu-baseline > "$R/gpurun_out/stats_head.log" 2>&1 || exit $?
echo "refresh done"
