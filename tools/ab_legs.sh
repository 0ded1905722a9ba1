#!/bin/bash
# A/B of the C3 / C5 / contended C5 legs between the default library and a variant build
# (multi-paxos_amd/lib_<variant>/libmpx.so, e.g. the previous sources), one process per
# leg and arm, alternating:  tools/ab_legs.sh <tag> <variant> [legs...]
set -o pipefail
tag=$1; var=$2; shift 2
legs=${@:-c3 c5 c5c}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for leg in $legs; do
  for arm in default $var; do
    envv=X=0; [ $arm != default ] && envv=MPX_LIB_VARIANT=$arm
    env $envv MPX_SIDE_PRIO=low timeout -k 10 300 python bench.py --$leg-only > $out/${leg}_$arm.json 2> $out/${leg}_$arm.err || { tail -20 $out/${leg}_$arm.err; exit 1; }
    python -c "
import json; d=json.loads(open('$out/${leg}_$arm.json').read().strip().splitlines()[-1]); k=list(d)[0]; c=d[k]
print('$leg', '$arm', round(c['ms_per_step'],4), {p: round(x, 4) for p, x in c['phases_ms'].items()}, c['counters_engine'] if 'counters_engine' in c else c['roofline'].get('counters_engine'), c.get('verified'))"
  done
done
