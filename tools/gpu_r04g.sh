set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MPX_LIB_VARIANT=q timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "(c3 or c5 or golden or kept_alternative or plan_path or member or decisions) and not full_size" > gpurun_out/r04_v9_tests_q.txt 2>&1 || { tail -40 gpurun_out/r04_v9_tests_q.txt; exit 1; }
tail -2 gpurun_out/r04_v9_tests_q.txt
bash tools/ab_c3.sh queue q noat || exit 2
