#!/bin/bash
# Round 6 closing run on the final commit (via gpurun): smoke + the GPU suite, the default bench line and
# the driver's command, then the rocprofv3 trace / HBM passes and the boundary leg (profiles/r6/final.sh).
set -o pipefail
OUT=${1:-gpurun_out/r6/final2}
bash profiles/r6/final.sh "$OUT" tests && bash profiles/r6/final.sh "$OUT" bench && bash profiles/r6/final.sh "$OUT" prof
