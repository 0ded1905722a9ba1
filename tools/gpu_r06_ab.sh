#!/bin/bash
# targeted GPU tests, then an A/B of two libraries over bench legs (tools/ab_legs.sh)
set -o pipefail
out=gpurun_out/${1:-r06_ab}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
shift 2
tools/ab_legs.sh "$@" || exit 2
