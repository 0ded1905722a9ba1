set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "incremental or kept_alternative or scan or engine_goldens or c3 or clean" > gpurun_out/r04_v2_tests.txt 2>&1 || { tail -30 gpurun_out/r04_v2_tests.txt; exit 1; }
tail -1 gpurun_out/r04_v2_tests.txt
bash tools/ab_shard_c4.sh ve ve || exit 2
bash tools/pmc_round.sh r04_v2 > gpurun_out/pmc_r04_v2.log 2>&1 || { tail -20 gpurun_out/pmc_r04_v2.log; exit 3; }
tail -5 gpurun_out/pmc_r04_v2.log
