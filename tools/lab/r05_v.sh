#!/bin/bash
# packed-ReLU tower check: eval-tower tests, tower timing against the previous
# tower (lab build) and the 32x32 scheduling variants, then the GPU suite,
# smoke and a bench line
set -o pipefail
R=gpurun_out/${VOUT:-r05v}; mkdir -p $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eval_head_gpu.py \
  > $R/tower_tests.log 2>&1 || exit 1
TWOUT=${VOUT:-r05v}/tw VARIANTS="${VARIANTS:-base old m32sep m32free}" bash tools/lab/r05_tw.sh || exit 1
timeout -k 10 700 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > $R/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $R/bench.json 2> $R/bench.err
