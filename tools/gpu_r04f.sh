set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "(c3 or c5 or golden or kept_alternative or plan_path or member or decisions) and not full_size" > gpurun_out/r04_v8_tests.txt 2>&1 || { tail -40 gpurun_out/r04_v8_tests.txt; exit 1; }
tail -3 gpurun_out/r04_v8_tests.txt
bash tools/ab_c3.sh side MPX_ONE_STREAM=1 noat || exit 2
