#!/bin/bash
# k_gate_votes A/B + the default bench (run under gpurun): member tests, the C5 / contended C5
# legs against lib_head, then the default bench line.
set -o pipefail
tag=${1:-r06_v}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "member or c5 or learn or epoch" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
bash tools/ab_legs.sh $tag head c5 c5c || exit 2
timeout -k 10 600 python bench.py --detail $out/bench_detail.json > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 3; }
grep "leg c\|C4:\|shard" $out/bench.err
