mkdir -p gpurun_out
for b in tools/lab_bin/ws_lab_*; do
  echo "== $b hb0"; timeout -k 5 60 $b 131072 512 512 5 1 0 || exit 1
  echo "== $b hb1"; timeout -k 5 60 $b 131072 512 512 5 0 1 || exit 1
done
