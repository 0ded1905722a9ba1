set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "(c3 or c5 or golden or kept_alternative or plan_path or member or decisions or store or clean) and not full_size" > gpurun_out/r04_v10_tests.txt 2>&1 || { tail -40 gpurun_out/r04_v10_tests.txt; exit 1; }
tail -2 gpurun_out/r04_v10_tests.txt
bash tools/ab_c3.sh xseg lseg4 || exit 2
