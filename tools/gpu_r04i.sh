set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MPX_LIB_VARIANT=pf1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "(c3 or golden or promise) and not full_size" > gpurun_out/r04_v12_tests_pf1.txt 2>&1 || { tail -30 gpurun_out/r04_v12_tests_pf1.txt; exit 1; }
tail -1 gpurun_out/r04_v12_tests_pf1.txt
bash tools/ab_c3.sh pf pf1 pf2 || exit 2
