#!/bin/bash
# targeted GPU tests, then the C3 windows leg alone (sequential and pipelined host loops)
set -o pipefail
out=gpurun_out/${1:-r06_w}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${2:-async_submit}" > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
timeout -k 10 600 python bench.py --c3-windows-only > $out/c3w.json 2> $out/c3w.err || { tail -20 $out/c3w.err; exit 3; }
grep "\[bench\]" $out/c3w.err
