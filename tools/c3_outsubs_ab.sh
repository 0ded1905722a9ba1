# C3 A/B of the snapshot sub-buffer count (MPX_OUT_SUBS, read at engine creation):
# one bench.py --c3-only process per arm on the same box
mkdir -p gpurun_out/c3subs
for k in 64 512 4096; do
  MPX_OUT_SUBS=$k timeout -k 10 400 python bench.py --c3-only > gpurun_out/c3subs/c3_$k.json 2> gpurun_out/c3subs/c3_$k.err || exit 1
done
