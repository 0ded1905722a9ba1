#!/bin/bash
# One GPU-box pass that produces a round's committed evidence (run under gpurun):
#   bench line, rocprofv3 kernel stats of the same command, PMC traffic for C4 and C3.
#   tools/gpu_profile.sh <tag>
set -o pipefail
tag=${1:-r02}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 420 python bench.py > $out/bench.json 2> $out/bench.err || exit 1
tail -c 400 $out/bench.json
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python bench.py --no-cpu-baseline > $out/prof.log 2>&1 || exit 2
python tools/kstats.py $(ls $out/prof/*_results.db | head -1) $out/kernel_stats.csv || exit 3
head -12 $out/kernel_stats.csv
timeout -k 10 600 python tools/pmc_traffic.py --tag ${tag}_c4 --outdir $out > $out/pmc_c4.log 2>&1 || exit 4
timeout -k 10 900 python tools/pmc_traffic.py --tag ${tag}_c3 --c3 --sq --outdir $out > $out/pmc_c3.log 2>&1 || exit 5
echo done
