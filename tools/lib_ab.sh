#!/bin/bash
# Kernel time of the kernels matching a name filter on one profile_paths path, for the product library and then every
# A/B library tools/probe/lib_*.so (built by tools/variant_build.sh): one rocprofv3 kernel trace per library.
# usage (gpurun, from the repo root): [REPS=n] bash tools/lib_ab.sh <name filter> <path>
set -o pipefail
F=$1; P=$2
R=$PWD
O=$R/gpurun_out/lib_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in product $(ls $R/tools/probe/lib_*.so 2>/dev/null); do
  if [ "$lib" = product ]; then t=product; unset SIREN_AMD_LIB; else t=$(basename $lib .so); export SIREN_AMD_LIB=$lib; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$t -o run -- python3 $R/tools/profile_paths.py $P --reps ${REPS:-5} > $O/$t.log 2>&1 || { echo "$t failed"; tail -5 $O/$t.log; exit 1; }
  python3 - "$O/$t" "$F" "$t" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)
for row in csv.DictReader(open(f[0])):
    if sys.argv[2] in row['Name']:
        print('%-14s %-40s calls %5s  avg %9.1f us  min %9.1f us' % (sys.argv[3], row['Name'][:40], row['Calls'],
              float(row['AverageNs']) / 1e3, float(row['MinNs']) / 1e3))
PY
done
