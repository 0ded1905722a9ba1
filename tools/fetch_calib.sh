#!/bin/bash
# FETCH_SIZE calibration for gather shapes (tools/fetch_probe.hip): the probe's
# known addresses, then one --pmc pass per counter group over the same binary:  tools/fetch_calib.sh <tag>
set -o pipefail
out=gpurun_out/${1:-fetch}
mkdir -p $out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O2 -o tools/fetch_probe tools/fetch_probe.hip || exit 9
timeout -k 10 60 tools/fetch_probe > $out/probe.jsonl || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fp --output-format csv -- tools/fetch_probe > $out/fetch.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $out/rdreq -o fp --output-format csv -- tools/fetch_probe > $out/rdreq.log 2>&1 || exit 3
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || exit 4
echo fetch-calib done
