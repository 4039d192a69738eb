# The distributed bench paths a one-GPU box can run (the N=8 run is the driver's):
#   1. one-rank RCCL group (WCE_FORCE_DIST=1): device broadcast, device barrier, max all-reduce
#   2. two ranks over gloo sharing GPU 0: the control path of the N>1 launch
# Outputs: gpurun_out/bench_forcedist.json, gpurun_out/bench_2rank_gloo.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
WCE_FORCE_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 \
    timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_forcedist.json 2> gpurun_out/bench_forcedist.err &&
WCE_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_2rank_gloo.json 2> gpurun_out/bench_2rank_gloo.err
