#!/bin/bash
# One or more legs of a PMC round (tools/pmc_traffic.py), each under its own time limit:
#   tools/pmc_part.sh <tag> c4|c3|c5|c5c|c3w ...
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for w in "$@"; do
  case $w in
    c4) args=""; lim=400 ;;
    c3) args="--c3 --sq"; lim=500 ;;
    c5) args="--c5"; lim=450 ;;
    c5c) args="--c5c"; lim=1000 ;;
    c3w) args="--c3w"; lim=500 ;;
    *) echo "unknown leg $w"; exit 9 ;;
  esac
  timeout -k 10 $lim python tools/pmc_traffic.py --tag ${tag}_$w $args > gpurun_out/pmc/${tag}_$w.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_$w.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pmc/${tag}_${w}_pmc.json')); print('$w', d['hbm_bytes_per_launch'], d['source_digest'])"
done
