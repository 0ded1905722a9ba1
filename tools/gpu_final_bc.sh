#!/bin/bash
# tools/gpu_final_b.sh then tools/gpu_final_c.sh in one call (run under gpurun):  tools/gpu_final_bc.sh <tag>
set -o pipefail
bash tools/gpu_final_b.sh ${1:-r06_final} && bash tools/gpu_final_c.sh ${1:-r06_final}
