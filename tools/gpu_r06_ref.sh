# round 6: REF PS_MMSE read-out forms (which 0: 0 = U1 nt, 3 = U1 plain, 4 = U2 nt,
# 5 = U4 nt, 1 = round 5's capped chunks), interleaved on the same buffers and
# bit-compared, beside PS_Linear alone on the same frames (same traffic shape)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_variants_gpu.py tests/test_parity_gpu.py -k "ref or variant" -m gpu > gpurun_out/ref_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 0 1 4 5 3 --frames 1048576 --rounds 5 --floor > gpurun_out/ab_ref_1m.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 0 1 4 5 --frames 65536 --rounds 5 --floor > gpurun_out/ab_ref_64k.txt 2>&1 &&
echo "r06 ref done"
