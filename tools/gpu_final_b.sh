#!/bin/bash
# Round-end evidence, part B: the default bench line and the rocprofv3 kernel stats of the
# same command.   tools/gpu_final_b.sh <tag>
set -o pipefail
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 3; }
tail -c 300 $out/bench.json
