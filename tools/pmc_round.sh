#!/bin/bash
# The PMC half of a measurement round (run under gpurun after tools/gpu_round.sh, same sources):
# HBM traffic of the C4, C3 (+ SQ wave states) and C5 apply phases, one rocprofv3 --pmc pass per
# counter group (tools/pmc_traffic.py):  tools/pmc_round.sh <tag>
set -o pipefail
tag=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 400 python tools/pmc_traffic.py --tag ${tag}_c4 > gpurun_out/pmc/${tag}_c4.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c4.log; exit 1; }
timeout -k 10 500 python tools/pmc_traffic.py --tag ${tag}_c3 --c3 --sq > gpurun_out/pmc/${tag}_c3.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c3.log; exit 2; }
timeout -k 10 400 python tools/pmc_traffic.py --tag ${tag}_c5 --c5 > gpurun_out/pmc/${tag}_c5.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c5.log; exit 3; }
timeout -k 10 600 python tools/pmc_traffic.py --tag ${tag}_c5c --c5c > gpurun_out/pmc/${tag}_c5c.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c5c.log; exit 5; }
timeout -k 10 500 python tools/pmc_traffic.py --tag ${tag}_c3w --c3w > gpurun_out/pmc/${tag}_c3w.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c3w.log; exit 4; }
for w in c4 c3 c5 c5c c3w; do python -c "import json; d=json.load(open('gpurun_out/pmc/${tag}_${w}_pmc.json')); print('$w', d['hbm_bytes_per_launch'], d['source_digest'])"; done
