#!/bin/bash
# Round profile on the GPU box: bench JSON line, rocprofv3 kernel trace+stats,
# and the two PMC passes (FETCH_SIZE / WRITE_SIZE) for HBM traffic.
# Usage (from the repo root, on the box): bash tools/profile_round.sh r01
set -o pipefail
R=${1:-r01}
OUT=gpurun_out/$R
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-serving --no-fp32 --no-zipf > $OUT/trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py --steps 3 --warmup 2 --eval-steps 1 --no-cpu-baseline --no-serving --no-fp32 --no-zipf > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
    python3 bench.py --steps 3 --warmup 2 --eval-steps 1 --no-cpu-baseline --no-serving --no-fp32 --no-zipf > $OUT/write.log 2>&1 &&
python3 tools/stats_summary.py $OUT/trace/run_kernel_stats.csv \
    "rocprofv3 --kernel-trace --stats of \`python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-serving --no-fp32 --no-zipf\`" \
    > $OUT/kernel_summary.txt &&
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv \
    --json $OUT/pmc_traffic.json > $OUT/pmc_traffic.txt &&
python3 tools/trace_passes.py $OUT/trace/run_kernel_trace.csv gemm_dw_kernel --per-step 9 \
    --warmup 5 --steps 20 > $OUT/gemm_dw_passes.txt &&
python3 tools/step_timeline.py $OUT/trace/run_kernel_trace.csv --step 12 --all > $OUT/step_timeline.txt
