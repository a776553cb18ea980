#!/bin/bash
# N=4 rehearsal of the bench's multi-rank path on one GPU (gloo; not a scaling figure)
set -o pipefail
mkdir -p gpurun_out
DCNR_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-serving --no-fp32 --no-zipf > gpurun_out/r05n4.json 2> gpurun_out/r05n4.err
