# C5 member apply A/B (bench.py --c5-only per arm): the default against
#   knob 524288 (k_apply walks every listed event, no-op E_EPOCH markers included)
#   knob 65536 (one k_apply over the whole work list, no AM_SIMPLE / AM_SNAP split)
mkdir -p gpurun_out/c5
timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5.json 2> gpurun_out/c5/c5.err || exit 1
MPX_KNOBS=524288 timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5_k524288.json 2> gpurun_out/c5/c5_k524288.err || exit 2
MPX_KNOBS=65536 timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5_k65536.json 2> gpurun_out/c5/c5_k65536.err || exit 3
