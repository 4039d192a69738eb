# round 5: four gloo ranks sharing GPU 0 -- bench.py's N>1 control path at N = 4 (the N=8 run is the driver's),
# plus the new small-batch ref_fc test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_framecov_gpu.py -m gpu > gpurun_out/fc_tests.log 2>&1 &&
WCE_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_4rank_gloo.json 2> gpurun_out/bench_4rank_gloo.err
