set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_part.sh r04_v13 c5 c3w || exit 1
MPX_LIB_VARIANT=prem timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "(c3 or c5 or golden or kept_alternative or plan_path or member or decisions or promise or fuzz) and not full_size" > gpurun_out/r04_v14_tests_prem.txt 2>&1 || { tail -30 gpurun_out/r04_v14_tests_prem.txt; exit 2; }
tail -1 gpurun_out/r04_v14_tests_prem.txt
bash tools/ab_c3.sh prem prem || exit 3
