#!/bin/bash
# Round 3, after the 3M apply: re-profile the legs whose kernels changed
# (apply = matvec_kernel at 65,536 frames, apply1m = apply_kernel at
# 1,048,576), merge them into the round's leg file, then the bench line and
# the rocprofv3 kernel statistics (tools/refresh_profiles.sh, SKIP_PMC=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R" && bash tools/pmc_legs.sh apply apply1m > "$R/gpurun_out/pmc_legs.log" 2>&1 || exit $?
python3 "$R/tools/pmc_merge.py" "$R/profiles/r03_pmc_legs.json" "$R/gpurun_out/pmc_legs.json" || exit $?
ROUND=r03 SKIP_PMC=1 bash "$R/tools/refresh_profiles.sh"
