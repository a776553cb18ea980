#!/bin/bash
# round 6: PMC ledger (FETCH_SIZE / WRITE_SIZE passes) of the train step for the
# default library and dW slab variants (tools/lab_bin/libdcnr_<v>.so)
#   bash tools/lab/r06_dw_pmc.sh <tag> "<variants>"
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/$1
A="--steps 3 --warmup 2 --eval-steps 1 --no-cpu-baseline --no-serving --no-fp32 --no-zipf"
for v in base $2; do
  O=$R/$v; mkdir -p $O
  if [ $v = base ]; then unset DCNR_LIB; else export DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so; fi
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- \
      python3 bench.py $A > $O/fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- \
      python3 bench.py $A > $O/write.log 2>&1 || exit 1
  python3 tools/pmc_ledger.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv \
      --bench $O/fetch.log > $O/ledger.txt || exit 1
done
