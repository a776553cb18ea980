# Same-box A/B of library builds on the cosine top-k (tools/knn_probe.py):
# the in-tree library and every tools/lab_bin/libdcnr_*.so, two rounds.
set -e
mkdir -p gpurun_out/abk
for r in 1 2; do
  timeout -k 10 120 python -u tools/knn_probe.py > gpurun_out/abk/base.$r.log 2>&1
  for so in tools/lab_bin/libdcnr_*.so; do
    n=$(basename $so .so)
    DCNR_LIB=$PWD/$so timeout -k 10 120 python -u tools/knn_probe.py > gpurun_out/abk/$n.$r.log 2>&1
  done
done
