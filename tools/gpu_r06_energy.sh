# round 6: configs[4] energy bound (tools/energy_bound.py), the REF leg's PMC passes
# (mmse_ref_elem_kernel), and the launcher-less two-rank rehearsal (bench.py --gpus 2, gloo)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/energy_bound.py --seconds 4 > gpurun_out/energy_bound.json 2> gpurun_out/energy_bound.err &&
timeout -k 10 400 bash tools/pmc_legs.sh ref > gpurun_out/pmc_ref.log 2>&1 &&
WCE_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
    --extras-out gpurun_out/bench_2rank_launcher_extras.json > gpurun_out/bench_2rank_launcher.json 2> gpurun_out/bench_2rank_launcher.err &&
echo "r06 energy done"
