# round 5: REF frame-covariance kernel rework -- its tests, then its legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_framecov_gpu.py tests/test_config5_ref_gpu.py tests/test_variants_gpu.py -m gpu > gpurun_out/gpu_fc.log 2>&1 &&
timeout -k 10 300 python -u tools/leg_time.py frame_cov config5_ref > gpurun_out/legs_fc.json 2> gpurun_out/legs_fc.err &&
timeout -k 10 300 python -u tools/ab_config5_streams.py > gpurun_out/ab_c5_streams.json 2> gpurun_out/ab_c5_streams.err
