#!/bin/bash
# k_plan_store8 A/B (run under gpurun): the C4-shaped GPU tests on the variant, then
# tools/ab_shard_c4.sh over the default library and the variants.
set -o pipefail
out=gpurun_out/r06_ps
mkdir -p $out
export TMPDIR=/tmp
sel="clean or golden or generator or store_chunks or c2_full or repeated or two_byte or wide or lookback"
MPX_LIB_VARIANT=${PS_TEST:-ps32} timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$sel" > $out/tests_ps.txt 2>&1 || { tail -30 $out/tests_ps.txt; exit 1; }
tail -1 $out/tests_ps.txt
bash tools/ab_shard_c4.sh ${AB_TAG:-r06_ps2} ${AB_ARMS:-ps16 ps24 ps32 ps40} || exit 2
