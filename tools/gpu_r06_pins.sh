# round 6: the COV mpmath pins on every solve form, the launcher-less two-rank bench test
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_cov_mp_gpu.py tests/test_textbook_mp_gpu.py tests/test_bench_launch.py -m gpu > gpurun_out/pins_tests.log 2>&1 &&
echo "r06 pins done"
