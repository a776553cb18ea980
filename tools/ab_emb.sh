set -e
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_embed_bwd_gpu.py tests/test_parity_gpu.py tests/test_stages_gpu.py tests/test_dp_gpu.py > gpurun_out/ab/t.log 2>&1
for r in 1 2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_old.so timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-serving --no-fp32 > gpurun_out/ab/old$r.log 2>&1
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-serving --no-fp32 > gpurun_out/ab/new$r.log 2>&1
done
