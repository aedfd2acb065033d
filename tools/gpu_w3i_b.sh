set -o pipefail
mkdir -p gpurun_out/w3i
timeout -k 10 300 python -u -m pytest tests/test_gpu_w3i.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w3i/tests2.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/w3i/tests2.log; exit 1; }
tail -1 gpurun_out/w3i/tests2.log
for p in ${PATHS:-w3_theta sdf}; do bash tools/gpu_variants.sh $p 4 || exit 1; done
