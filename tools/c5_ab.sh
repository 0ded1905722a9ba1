# C5 member apply A/B: the three-way split (default) against one kernel (knob 65536)
# and no AM_SNAP kernel (knob 262144)
mkdir -p gpurun_out/c5
timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5.json 2> gpurun_out/c5/c5.err || exit 1
MPX_KNOBS=65536 timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5_k65536.json 2> gpurun_out/c5/c5_k65536.err || exit 2
MPX_KNOBS=262144 timeout -k 10 500 python bench.py --c5-only --c5-instances 33554432 > gpurun_out/c5/c5_k262144.json 2> gpurun_out/c5/c5_k262144.err || exit 3
