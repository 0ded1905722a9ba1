#!/bin/bash
# The C5, contended C5 and C3-windows PMC passes (run under gpurun):  tools/gpu_final_c.sh <tag>
set -o pipefail
tag=${1:-r06_final}
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 400 python tools/pmc_traffic.py --tag ${tag}_c5 --c5 > gpurun_out/pmc/${tag}_c5.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c5.log; exit 3; }
timeout -k 10 600 python tools/pmc_traffic.py --tag ${tag}_c5c --c5c > gpurun_out/pmc/${tag}_c5c.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c5c.log; exit 5; }
timeout -k 10 500 python tools/pmc_traffic.py --tag ${tag}_c3w --c3w > gpurun_out/pmc/${tag}_c3w.log 2>&1 || { tail -20 gpurun_out/pmc/${tag}_c3w.log; exit 4; }
for w in c5 c5c c3w; do python -c "import json; d=json.load(open('gpurun_out/pmc/${tag}_${w}_pmc.json')); print('$w', d['hbm_bytes_per_launch'], d['source_digest'])"; done
