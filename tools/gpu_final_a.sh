#!/bin/bash
# Round-end evidence, part A (under gpurun): every GPU test (full-size ones printing their
# progress), smoke, the default bench line.   tools/gpu_final_a.sh <tag>
set -o pipefail
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 900 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit 2
