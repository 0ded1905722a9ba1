# C5 A/B of the k_chosen grid (MPX_CHOSEN_WGS_PER_CU; member walks every bucket's chosen list)
mkdir -p gpurun_out/c5ch
for k in 4 8 16; do
  MPX_CHOSEN_WGS_PER_CU=$k timeout -k 10 400 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5ch/c5_$k.json 2> gpurun_out/c5ch/c5_$k.err || exit 1
done
