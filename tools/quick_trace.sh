#!/bin/bash
# Kernel-time A/B after a kernel edit: for each path, one HIP-event timing run and one rocprofv3 kernel trace
# (no PMC), then the per-kernel averages of the kernels matching $KFILTER (default: all) are printed.
# usage (gpurun, from the repo root): [KFILTER=wgrad] bash tools/quick_trace.sh <tag> <paths...>
set -o pipefail
TAG=$1
shift
R=$PWD
O=$R/gpurun_out/qt_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for p in "$@"; do
  mkdir -p $O/$p
  timeout -k 10 120 python3 $R/tools/profile_paths.py $p > $O/$p/timing.json 2> $O/$p/timing.err || { echo "timing $p failed"; tail -5 $O/$p/timing.err; exit 1; }
  cat $O/$p/timing.json
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$p/trace -o run -- python3 $R/tools/profile_paths.py $p > $O/$p/trace.log 2>&1 || { echo "trace $p failed"; tail -5 $O/$p/trace.log; exit 1; }
  python3 - "$O/$p/trace" "${KFILTER:-}" <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)
for row in csv.DictReader(open(f[0])):
    if sys.argv[2] in row['Name']:
        print('   %-40s calls %5s  avg %9.1f us' % (row['Name'][:40], row['Calls'], float(row['AverageNs']) / 1e3))
EOF
done
