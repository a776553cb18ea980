#!/bin/bash
# SQ counter passes over one lab binary (on the GPU box, from the repo root):
#   bash tools/pmc_lab.sh <binary> <out-dir> [args...]
set -o pipefail
export TMPDIR=/tmp
B=$1; O=$2; shift 2
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
P2="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_BANK_CONFLICT"
P3="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SALU SQ_WAVES"
mkdir -p $O
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$i -o run -- $B "$@" > $O/p$i.log 2>&1 || exit 1
done
