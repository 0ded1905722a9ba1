set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_c3.sh waves2 w5 w6 w5s || exit 2
