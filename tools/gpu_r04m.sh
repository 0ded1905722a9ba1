#!/bin/bash
# Plan-list window restaging: the full-size oracle checks, the goldens, then the leg A/B against
# the previous sources (lib_old):  tools/gpu_r04m.sh <tag>
set -o pipefail
T=${1:-r04_vX}
out=gpurun_out/$T
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v -s --timeout 600 --timeout-method thread \
  -k "full_size or golden or commit_value or violations or contended_2_20" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
bash tools/ab_legs.sh $T old c3 c5 c5c
