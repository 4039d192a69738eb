#!/bin/bash
# Copy what tools/refresh_profiles.sh left in gpurun_out/ into profiles/ under
# this round's names.  usage: tools/collect_profiles.sh [r02]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
RND=${1:-r02}
G=$R/gpurun_out
cp "$G/bench_full.json" "$R/profiles/${RND}_bench.json"
cp "$G/stats/run_kernel_stats.csv" "$R/profiles/${RND}_kernel_stats.csv"
[ -f "$G/stats_head/run_kernel_stats.csv" ] && cp "$G/stats_head/run_kernel_stats.csv" "$R/profiles/${RND}_kernel_stats_headline.csv"
[ -f "$G/pmc_legs.json" ] && cp "$G/pmc_legs.json" "$R/profiles/${RND}_pmc_legs.json"
echo "collected into profiles/ as ${RND}_*"
