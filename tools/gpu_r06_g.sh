#!/bin/bash
# Gather change A/B (run under gpurun): the plan-path GPU tests on the default library, then
# the C3 / C5 / contended C5 legs and the C4 step / shard against lib_head (the previous sources).
set -o pipefail
tag=${1:-r06_g1}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${SEL:-c3 or c5 or golden or member or plan or clean}" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
bash tools/ab_legs.sh $tag head ${LEGS:-c3 c5 c5c} || exit 2
bash tools/ab_legs.sh ${tag}b head ${LEGS2:-c3 c5c} || exit 3
[ -z "$SKIP_C4" ] && { bash tools/ab_shard_c4.sh $tag head || exit 4; }
true
