#!/bin/bash
# GPU parity pass: optional focused test files first (args), then the whole -m gpu suite; logs under gpurun_out/<tag>.
# usage (gpurun, from the repo root): bash tools/gpu_tests.sh <tag> [test files...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $O/focus.log 2>&1; rc=$?
  tail -5 $O/focus.log
  [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
exit $rc
