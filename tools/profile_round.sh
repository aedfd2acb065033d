#!/bin/bash
# Per-path profiles of the training / inference kernels (tools/profile_paths.py): for every path one HIP-event
# timing run, one rocprofv3 kernel-trace + stats run, and two PMC passes (FETCH_SIZE, WRITE_SIZE: one counter group
# per pass, never combined with tracing), then tools/path_summary.py -> <out>/pmc_<path>.json.
# usage (gpurun, from the repo root): [SQ_PASSES=1] bash tools/profile_round.sh <tag> [paths...]
# SQ_PASSES=1 adds three SQ counter passes (wave / wait cycles, MFMA / VALU busy and instruction counts, LDS).
set -o pipefail
TAG=${1:-r02}
shift
PATHS_TO_RUN=${@:-"w1 image_w2 sdf w3_theta w3_wide video video1024 poisson poisson_ref hypernet"}
R=$PWD
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for p in $PATHS_TO_RUN; do
  mkdir -p $O/$p
  timeout -k 10 120 python3 $R/tools/profile_paths.py $p > $O/$p/timing.json 2> $O/$p/timing.err || { echo "timing $p failed"; tail -5 $O/$p/timing.err; exit 1; }
  cat $O/$p/timing.json
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$p/trace -o run -- python3 $R/tools/profile_paths.py $p > $O/$p/trace.log 2>&1 || { echo "trace $p failed"; tail -5 $O/$p/trace.log; exit 1; }
  i=0
  PASSLIST="FETCH_SIZE WRITE_SIZE"
  if [ -n "$SQ_PASSES" ]; then PASSLIST="$PASSLIST SQA SQB SQC"; fi
  for grp in $PASSLIST; do
    case $grp in
      SQA) grp="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE";;
      SQB) grp="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU";;
      SQC) grp="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM";;
    esac
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/$p/pmc$i -o pmc -- python3 $R/tools/profile_paths.py $p > $O/$p/pmc$i.log 2>&1 || { echo "pmc $grp $p failed"; exit 1; }
  done
done
cd $R && python3 tools/path_summary.py $O $O && echo done
