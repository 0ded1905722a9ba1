#!/bin/bash
# One stream vs the side stream for member legs (MPX_ONE_STREAM), alternating arms:  tools/ab_member_stream.sh <tag>
set -o pipefail
T=${1:-r04_vX}
out=gpurun_out/$T
mkdir -p $out
export TMPDIR=/tmp
run() { name=$1; leg=$2; shift 2; env "$@" timeout -k 10 240 python bench.py --$leg-only > $out/$name.json 2> $out/$name.err || { tail -20 $out/$name.err; exit 2; }
  python -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); c=list(d.values())[0]
print('$name', round(c['ms_per_step'],4), {p: round(x, 4) for p, x in c['phases_ms'].items()}, c['verified']['step_state_digest_vs_run'])"; }
run c5c_side c5c X=0
run c5c_one c5c MPX_ONE_STREAM=1
run c5_side c5 X=0
run c5_one c5 MPX_ONE_STREAM=1
run c5c_side2 c5c X=0
run c5c_one2 c5c MPX_ONE_STREAM=1
