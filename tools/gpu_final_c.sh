#!/bin/bash
# Round-end evidence, part C: rocprofv3 kernel stats of the bench command (no CPU baseline).
set -o pipefail
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python bench.py --no-cpu-baseline > $out/prof.log 2>&1 || exit 4
python tools/kstats.py $(ls $out/prof/*_results.db $out/prof/*/*_results.db 2>/dev/null | head -1) $out/kernel_stats.csv || exit 5
head -25 $out/kernel_stats.csv
