# C4-only kernel stats, default launch vs the header kernels as three launches (knob 134217728)
export TMPDIR=/tmp
mkdir -p gpurun_out/c4split
for arm in default split; do
  if [ $arm = split ]; then export MPX_KNOBS=134217728; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4split/$arm -o c4 -- python bench.py --no-cpu-baseline --c3-instances 0 --c5-instances 0 --shard-of 0 --steps 20 > gpurun_out/c4split/$arm.log 2>&1 || exit 1
  python tools/kstats.py $(ls gpurun_out/c4split/$arm/*_results.db gpurun_out/c4split/$arm/*/*_results.db 2>/dev/null | head -1) gpurun_out/c4split/$arm.csv || exit 2
  head -12 gpurun_out/c4split/$arm.csv | cut -d, -f1-4
done
