#!/bin/bash
# Member A/B: the 8-segment member plan (lib_m8) and one stream (MPX_ONE_STREAM) on C5 / contended C5,
# plus the member GPU tests on the variant:  tools/gpu_r04l.sh <tag>
set -o pipefail
T=${1:-r04_vX}
out=gpurun_out/$T
mkdir -p $out
export TMPDIR=/tmp
MPX_LIB_VARIANT=m8 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q -s --timeout 600 --timeout-method thread -k "member or c5" > $out/tests_m8.txt 2>&1 || { tail -30 $out/tests_m8.txt; exit 1; }
tail -1 $out/tests_m8.txt
run() { name=$1; leg=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --$leg-only > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 2; }
  python -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); c=list(d.values())[0]
print('$name', round(c['ms_per_step'],4), {p: round(x, 4) for p, x in c['phases_ms'].items()}, c['roofline']['counters_engine']['general_pairs'], c['verified']['step_state_digest_vs_run'])"; }
run c5_default c5 X=0
run c5_m8 c5 MPX_LIB_VARIANT=m8
run c5_one c5 MPX_ONE_STREAM=1
run c5c_default c5c X=0
run c5c_m8 c5c MPX_LIB_VARIANT=m8
run c5c_one c5c MPX_ONE_STREAM=1
run c5c_m8_one c5c MPX_LIB_VARIANT=m8 MPX_ONE_STREAM=1
