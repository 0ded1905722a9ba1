#!/bin/bash
# A/B of the side stream's priority (MPX_SIDE_PRIO) inside the bench's own process order
# (C4 engine, shard engine, then the C3 leg), plus the C3 leg alone:  tools/ab_side_prio.sh <tag>
set -o pipefail
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for arm in normal low high; do
  MPX_SIDE_PRIO=$arm timeout -k 10 300 python bench.py --no-cpu-baseline --c5-instances 0 --c5c-instances 0 --c3-windows 0 \
    > $out/side_$arm.json 2> $out/side_$arm.err || { tail -20 $out/side_$arm.err; exit 1; }
  python -c "import json; d=json.loads(open('$out/side_$arm.json').read().strip().splitlines()[-1]); print('$arm', 'c4', round(d['ms_per_step'],4), 'shard', round(d['scaling_projection']['T_shard_ms'],4), 'c3', round(d['c3']['ms_per_step'],4), d['c3'].get('verified'))"
done
for arm in normal low; do
  MPX_SIDE_PRIO=$arm timeout -k 10 200 python bench.py --c3-only > $out/side_c3only_$arm.json 2> $out/side_c3only_$arm.err || exit 2
  python -c "import json; d=json.loads(open('$out/side_c3only_$arm.json').read().strip().splitlines()[-1]); c=d.get('c3',d); print('c3-only $arm', round(c['ms_per_step'],4))"
done
