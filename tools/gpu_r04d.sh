set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=25 \
  -k "not full_size" > gpurun_out/r04_v5_tests.txt 2>&1 || { tail -40 gpurun_out/r04_v5_tests.txt; exit 1; }
tail -30 gpurun_out/r04_v5_tests.txt
bash tools/ab_shard_env.sh scan MPX_SCAN_SMALL=0 || exit 2
bash tools/ab_c3.sh rows rows || exit 3
