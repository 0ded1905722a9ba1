#!/bin/bash
# GPU tests + smoke + the default bench line (run under gpurun):  tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
tag=${1:-r06}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -n "$2" ]; then sel=(-k "$2"); else sel=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${sel[@]}" > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -1 $out/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { cat $out/smoke.txt; exit 2; }
timeout -k 10 900 python bench.py --detail $out/bench_detail.json > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 3; }
cat $out/bench.err | grep -v "^\[bench\] c[35c]*: \(generated\|ingested\|upload\)"
