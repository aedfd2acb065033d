#!/bin/bash
# One GPU-box pass: parity suite, default bench line, rocprofv3 kernel stats of the bench, PMC HBM passes.
# usage (gpurun, from the repo root): bash tools/gpu_round.sh <tag> [skip_tests]
set -o pipefail
TAG=${1:-r01}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "$2" != "skip_tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --no-extra --no-dp --steps 10 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc/pass$i -o pmc -- python3 $R/bench.py --no-cpu --no-extra --no-dp --steps 5 > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
cd $R && python tools/pmc_summary.py $O/pmc 1048576 $O/pmc.json && echo done
