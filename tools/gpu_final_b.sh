#!/bin/bash
# Kernel stats of the default bench command + the C4 and C3 PMC passes (run under gpurun):
#   tools/gpu_final_b.sh <tag>
set -o pipefail
tag=${1:-r06_final}
out=gpurun_out/$tag
mkdir -p $out gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python bench.py --no-cpu-baseline > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 4; }
python tools/kstats.py $(ls $out/prof/*_results.db $out/prof/*/*_results.db 2>/dev/null | head -1) $out/kernel_stats.csv || exit 5
head -25 $out/kernel_stats.csv
timeout -k 10 400 python tools/pmc_traffic.py --tag ${tag}_c4 > gpurun_out/pmc/${tag}_c4.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c4.log; exit 1; }
timeout -k 10 500 python tools/pmc_traffic.py --tag ${tag}_c3 --c3 --sq > gpurun_out/pmc/${tag}_c3.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c3.log; exit 2; }
for w in c4 c3; do python -c "import json; d=json.load(open('gpurun_out/pmc/${tag}_${w}_pmc.json')); print('$w', d['hbm_bytes_per_launch'], d['source_digest'])"; done
