# Same-box A/B of library builds: bench.py (headline step, no extra legs)
# with DCNR_LIB pointing at each tools/lab_bin/libdcnr_*.so and the in-tree
# library, two rounds.  Usage on the box: bash tools/ab_variants.sh
set -e
mkdir -p gpurun_out/abv
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-serving --no-fp32 --no-zipf > gpurun_out/abv/base$r.log 2>&1
  for so in tools/lab_bin/libdcnr_*.so; do
    n=$(basename $so .so)
    DCNR_LIB=$PWD/$so timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-serving --no-fp32 --no-zipf > gpurun_out/abv/$n.$r.log 2>&1
  done
done
