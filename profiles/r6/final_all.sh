#!/bin/bash
# Round 6 closing run on the final commit (via gpurun), in two calls of <= 20 minutes:
#   A: smoke + the GPU suite, the default bench line and the driver's command;
#   B: the rocprofv3 trace / HBM passes, the boundary leg and the multi-rank rehearsal.
set -o pipefail
OUT=${1:-gpurun_out/r6/final2}
case ${2:-A} in
  A) bash profiles/r6/final.sh "$OUT" tests && bash profiles/r6/final.sh "$OUT" bench ;;
  B) bash profiles/r6/final.sh "$OUT" prof ;;
esac
