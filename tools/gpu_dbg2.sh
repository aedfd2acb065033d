set -o pipefail
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -u -m pytest tests/test_gpu_w3i.py -q --timeout 200 --timeout-method thread -k grouped > gpurun_out/dbg/grouped.log 2>&1; echo "rc $?"; grep -E "Error|passed|failed" gpurun_out/dbg/grouped.log | head -20
