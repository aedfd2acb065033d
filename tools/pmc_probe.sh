#!/bin/bash
# Extra PMC passes over the W1 bench (instruction cache, LDS, barrier/wait breakdown). usage: bash tools/pmc_probe.sh <outdir>
R=$PWD
O=$R/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
i=0
for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pass$i -o pmc -- python3 $R/bench.py --no-cpu --no-extra --steps 3 --warmup 1 > $O/pass$i.log 2>&1 || echo "pass $i failed: $grp" >> $O/failures.txt
done
cd $R && python tools/pmc_summary.py $O 1048576 $O/summary.json
