# quick check: accuracy tests + headline bench (+ optional extra pytest args in $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_accuracy_gpu.py ${EXTRA_TESTS} -m gpu > gpurun_out/quick_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err
