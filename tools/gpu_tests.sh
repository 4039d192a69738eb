# the round-end GPU gate, as the driver runs it: pytest -m gpu, then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
