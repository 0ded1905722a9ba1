set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 \
  -k "member or mm_ or c5_ or decisions or learns or incremental or propose" > gpurun_out/r04_v4_tests.txt 2>&1 || { tail -40 gpurun_out/r04_v4_tests.txt; exit 1; }
tail -20 gpurun_out/r04_v4_tests.txt
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -v -s --timeout-method thread \
  -k "c5_contended_full_size or c5_full_size" > gpurun_out/r04_v4_full.txt 2>&1 || { tail -40 gpurun_out/r04_v4_full.txt; exit 2; }
tail -8 gpurun_out/r04_v4_full.txt
