#!/bin/bash
# A/B of library variants on the GPU box: for each gpurun_exp/lib_<tag>.so, install it as siren_amd/libsiren_amd.so
# and run tools/time_split.py (and the split parity tests when AB_TESTS=1); the original library is restored at the end.
set -o pipefail
R=$PWD
cp siren_amd/libsiren_amd.so /tmp/lib_orig_backup.so
for f in gpurun_exp/lib_*.so; do
  tag=$(basename $f .so)
  cp $f siren_amd/libsiren_amd.so
  echo "== $tag"
  if [ -n "$AB_TESTS" ]; then
    timeout -k 10 200 python -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || { cp /tmp/lib_orig_backup.so siren_amd/libsiren_amd.so; exit 1; }
  fi
  timeout -k 10 120 python tools/time_split.py --reps 30 2>&1 | tail -1 || { cp /tmp/lib_orig_backup.so siren_amd/libsiren_amd.so; exit 1; }
done
cp /tmp/lib_orig_backup.so siren_amd/libsiren_amd.so
