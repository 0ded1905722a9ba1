#!/bin/bash
# Window-kernel / member-walk gather A/B (run under gpurun): targeted tests, the C3-windows leg
# with each library twice (arms alternated), then the contended C5 and C3 legs (tools/ab_legs.sh).
set -o pipefail
tag=${1:-r06_w2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "incremental or window or member or c5 or golden" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for rep in 1 2; do
  for arm in default head; do
    envv=X=0; [ $arm != default ] && envv=MPX_LIB_VARIANT=$arm
    env $envv timeout -k 10 300 python bench.py --c3-windows-only > $out/w_${arm}_$rep.json 2> $out/w_${arm}_$rep.err || { tail -20 $out/w_${arm}_$rep.err; exit 2; }
    echo "$arm $rep $(grep -o 'k_apply_win [0-9.]* ms' $out/w_${arm}_$rep.err | head -1) $(grep -o 'device [0-9.]*' $out/w_${arm}_$rep.err | head -1)"
  done
done
bash tools/ab_legs.sh $tag head c5c c3 || exit 3
