#!/bin/bash
# SQ / SQC counters of the fused eval tower (tools/tower_probe.py at B=131072),
# one rocprofv3 --pmc pass each.   bash tools/tower_counters.sh <tag>
set -o pipefail
R=${1:-r04}
OUT=gpurun_out/$R/twsq
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P3="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE"
# L2: hit rate of the weight stream, memory-side reads (Infinity Cache or HBM)
P4="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/$OUT/p$i -o run -- \
      python3 $ROOT/tools/tower_probe.py 131072 > $ROOT/$OUT/p$i.log 2>&1) || echo "pass $i failed" >> $ROOT/$OUT/status.txt
done
python3 tools/sq_summary.py $OUT > gpurun_out/$R/tower_counters.txt 2>&1 || true
