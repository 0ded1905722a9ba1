set -o pipefail
out=gpurun_out/r04_v1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "incremental or kept_alternative or member_plan_path" > $out/targeted.txt 2>&1 || { tail -40 $out/targeted.txt; exit 1; }
tail -2 $out/targeted.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail 20 > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 2; }
tail -2 $out/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit 3
timeout -k 10 420 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 4; }
tail -c 400 $out/bench.json
