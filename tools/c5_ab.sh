mkdir -p gpurun_out/c5
timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5.json 2> gpurun_out/c5/c5.err || exit 1
MPX_APPLY_VARIANT=1 timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5_v1.json 2> gpurun_out/c5/c5_v1.err || exit 2
