# round 4: PMC legs in parts (one gpurun call each; LEGS="..." selects the part)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 1100 bash tools/pmc_legs.sh $LEGS > gpurun_out/pmc_legs.log 2>&1
