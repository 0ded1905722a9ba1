#!/bin/bash
# One GPU-box pass: the GPU tests, smoke, the default bench line and the rocprofv3
# kernel stats of the same bench command (run under gpurun):  tools/gpu_round.sh <tag>
set -o pipefail
tag=${1:-r03}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 900 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit 2
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 3; }
tail -c 300 $out/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python bench.py --no-cpu-baseline > $out/prof.log 2>&1 || exit 4
python tools/kstats.py $(ls $out/prof/*_results.db $out/prof/*/*_results.db 2>/dev/null | head -1) $out/kernel_stats.csv || exit 5
head -25 $out/kernel_stats.csv
