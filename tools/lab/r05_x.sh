#!/bin/bash
# round 5: ragged top-k shapes, the sparse exchange's row-map step (two ranks
# on one GPU), then the N=2 rehearsal line with the exchange window
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py tests/test_dp_gpu.py tests/test_row_map_gpu.py \
  -k "small_and_ragged or sparse_exchange or row_map or step_rows" > gpurun_out/r05x_tests.log 2>&1 || exit 1
DCNR_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  --no-cpu-baseline --no-serving --no-fp32 --no-zipf > gpurun_out/r05x_n2.json 2> gpurun_out/r05x_n2.err
