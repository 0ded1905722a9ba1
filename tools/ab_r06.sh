#!/bin/bash
# Round-6 measurements (run under gpurun): the host window cost on the box's CPUs (ingest_bench:
# decode / build per window, no GPU), then the C3 leg A/B of k_plan_list's staging variants
set -o pipefail
out=gpurun_out/${1:-ab_r06}
mkdir -p $out
MPX_DECODE_TIMES=1 MPX_BUILD_TIMES=1 timeout -k 10 300 tools/ingest_bench 24 16 > $out/ingest_bench.txt 2>&1 || { tail -5 $out/ingest_bench.txt; exit 1; }
grep -E "per window|window 15" $out/ingest_bench.txt
grep "\[mpx\]" $out/ingest_bench.txt | tail -4
tools/ab_c3.sh pl k16 f32 || exit 2
