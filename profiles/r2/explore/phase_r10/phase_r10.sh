#!/bin/bash
# r2: phase split of the final kernel with the rank accumulation (run 10)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-phase_r10}; mkdir -p $O
PHASE_ARGS="c2 0 8 15" bash profiles/phase_variants.sh $O phase && mv $O/phase.log $O/phase_c2.log \
 && PHASE_ARGS="c3 0" bash profiles/phase_variants.sh $O phase && mv $O/phase.log $O/phase_c3.log
