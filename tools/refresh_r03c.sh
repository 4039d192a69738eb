#!/bin/bash
# Round 3, after the low-rank lane kernel changes (P_k / U shared in LDS, the
# staged form at every size): GPU gate, re-profile the lowrank4 / lowrank8 PMC
# legs, merge them into the round's leg file, then the bench line and the
# rocprofv3 kernel statistics (tools/refresh_profiles.sh, SKIP_PMC=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R" && timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > "$R/gpurun_out/gpu_tests.log" 2>&1 || exit $?
bash tools/pmc_legs.sh lowrank4 lowrank8 > "$R/gpurun_out/pmc_legs.log" 2>&1 || exit $?
python3 "$R/tools/pmc_merge.py" "$R/profiles/r03_pmc_legs.json" "$R/gpurun_out/pmc_legs.json" || exit $?
ROUND=r03 SKIP_PMC=1 bash "$R/tools/refresh_profiles.sh"
