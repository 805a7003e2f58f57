#!/bin/bash
# Round 3 run 2 (via gpurun): the GPU suite (scene BVH, boundary, sharded gather) and C2 benches, then
# explore1 (beam-key study, sqrt-mode stakes, full-size C4).
set -o pipefail
OUT=${1:-gpurun_out/r3/run2}
bash profiles/r3/suite.sh "$OUT" skip_c4 && bash profiles/r3/explore1.sh "$OUT/explore1"
