#!/bin/bash
# time one profile_paths path for the default library (flags 0 and SIREN_FLAGS=$ALT) and every tools/probe/lib_*.so
# usage (gpurun): bash tools/gpu_variants.sh <path> [alt_flags]
set -o pipefail
P=${1:-w3_theta}; ALT=${2:-4}
mkdir -p gpurun_out/var
for f in 0 $ALT; do
  SIREN_FLAGS=$f timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/base_$f.json 2> gpurun_out/var/base_$f.err || { echo "base $f failed"; tail -5 gpurun_out/var/base_$f.err; exit 1; }
  echo "base flags=$f $(cat gpurun_out/var/base_$f.json)"
done
for lib in $(ls tools/probe/lib_*.so 2>/dev/null); do
  t=$(basename $lib .so)
  SIREN_AMD_LIB=$lib timeout -k 10 120 python tools/profile_paths.py $P > gpurun_out/var/$t.json 2> gpurun_out/var/$t.err || { echo "$t failed"; tail -5 gpurun_out/var/$t.err; exit 1; }
  echo "$t $(cat gpurun_out/var/$t.json)"
done
