set -o pipefail
mkdir -p gpurun_out/dbg
for f in 4 0; do
SIREN_TEST_FLAGS=$f timeout -k 10 300 python -u -m pytest -p tools.flags_plugin tests/test_gpu_batched.py -x -q -s --timeout 200 --timeout-method thread -k "second_and_third" > gpurun_out/dbg/batched_$f.log 2>&1; echo "flags $f rc $?"; grep -E "rel|passed|failed" gpurun_out/dbg/batched_$f.log | head -5
done
