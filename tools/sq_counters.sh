#!/bin/bash
# SQ (shader sequencer) counters of the production kernels: MFMA-busy, LDS
# issue stalls and bank conflicts, wave states.  Two PMC passes over the same
# short bench.py run (8 SQ + 1 GRBM counters each), then tools/sq_summary.py
# reduces them per kernel.  On the GPU box, from the repo root:
#   bash tools/sq_counters.sh r03a
# SQ_PROG overrides the program (default: a short bench.py run), e.g.
#   SQ_PROG="tools/knn_lab.py" bash tools/sq_counters.sh r03q
set -o pipefail
R=${1:-r03}
OUT=gpurun_out/$R/sq
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --eval-steps 1 --no-cpu-baseline --no-serving --no-fp32 --no-zipf"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 ${SQ_PROG:-bench.py $ARGS} > $OUT/p$i.log 2>&1 || exit 1
done
python3 tools/sq_summary.py $OUT > gpurun_out/$R/sq_counters.txt
