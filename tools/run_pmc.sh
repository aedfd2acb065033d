#!/bin/bash
# rocprofv3 PMC passes over the W1 bench (one counter group per pass; never combined with tracing domains).
# usage (on the GPU box, from the repo root): bash tools/run_pmc.sh <outdir> [bench args...]
set -e
OUT=$1; shift
R=$PWD
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/$OUT/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $R/$OUT/pass$i -o pmc -- python3 $R/bench.py "$@" > $R/$OUT/pass$i.log 2>&1 || echo "pass $i failed: $grp" >> $R/$OUT/failures.txt
done
