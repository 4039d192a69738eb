set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/quick_lowrank.py > gpurun_out/quick_lowrank.json 2>&1
