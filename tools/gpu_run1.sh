set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_accuracy_gpu.py -m gpu -s > gpurun_out/acc_tests.log 2>&1
echo "acc rc=$?"
timeout -k 10 120 python -u tools/accuracy_probe.py > gpurun_out/acc_probe.txt 2>&1 &&
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1
echo "rc=$?"
