#!/bin/bash
# Kernel time of one kernel (name filter $1) on one profile_paths path ($2) for each probe library tools/probe/lib_*.so
# (and the product library): rocprofv3 kernel trace per library. usage (gpurun): bash tools/probe_trace.sh <filter> <path>
set -o pipefail
F=$1; P=$2
R=$PWD
O=$R/gpurun_out/probe_trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in $(ls $R/tools/probe/lib_*.so) $(ls $R/tools/probe/lib_*.so); do
  t=$(basename $lib .so); [ -d $O/$t ] && t=${t}_2
  if [ "$lib" = product ]; then unset SIREN_AMD_LIB; else export SIREN_AMD_LIB=$lib; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$t -o run -- python3 $R/tools/profile_paths.py $P > $O/$t.log 2>&1 || { echo "$t failed"; tail -5 $O/$t.log; exit 1; }
  python3 - "$O/$t" "$F" "$t" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)
for row in csv.DictReader(open(f[0])):
    if sys.argv[2] in row['Name']:
        print('%-14s %-40s calls %5s  avg %9.1f us' % (sys.argv[3], row['Name'][:40], row['Calls'], float(row['AverageNs']) / 1e3))
PY
done
