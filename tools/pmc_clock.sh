#!/bin/bash
# Effective clock and MFMA-busy of one lab binary's kernel under rocprofv3 PMC
# (GRBM_GUI_ACTIVE / 8 / duration; SQ_VALU_MFMA_BUSY_CYCLES / (1024 x that)):
#   bash tools/pmc_clock.sh <out-dir> <binary> [args...]
set -o pipefail
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O -o run -- "$@" \
    > $O/run.log 2>&1
