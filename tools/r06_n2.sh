#!/bin/bash
# round 6: the bench's N>1 path rehearsed on one GPU (both ranks on cuda:0 over
# gloo; not a scaling number) and the world-2 DP tests
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dp_gpu.py > $R/dp_tests.log 2>&1 || exit 1
tail -n 1 $R/dp_tests.log
DCNR_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  --no-cpu-baseline --no-serving --no-fp32 --no-zipf > $R/n2.json 2> $R/n2.err || exit 1
python3 -c "import json;d=json.loads(open('$R/n2.json').read().strip().splitlines()[-1]);print(json.dumps({k: d[k] for k in ('n_gpus','value','ms_per_step','distributed','exchange_window_after_backward')})); print(d['config'])"
