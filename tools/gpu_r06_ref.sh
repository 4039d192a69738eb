# round 6: REF PS_MMSE read-out forms (which 0: 0 = U1 nt 256 threads, 6 / 7 / 8 = 512 /
# 1024 / 128 threads, 1 = round 5's capped chunks), interleaved on the same buffers
# and bit-compared, at batch sizes around the MALL
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_variants_gpu.py -m gpu > gpurun_out/ref_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 0 6 7 8 1 --frames 1048576 --rounds 5 > gpurun_out/ab_ref_1m.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 0 1 --frames 262144 --rounds 5 > gpurun_out/ab_ref_256k.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 0 1 --frames 131072 --rounds 5 > gpurun_out/ab_ref_128k.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_variant.py ref --variants 0 6 1 --frames 65536 --rounds 5 > gpurun_out/ab_ref_64k.txt 2>&1 &&
echo "r06 ref done"
