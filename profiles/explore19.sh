#!/bin/bash
# r2: phase split of the current production kernel (no-SLP, squared prefilter, transposed scan, occupancy 7)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore19}; mkdir -p $O
PHASE_ARGS="c2 0 8 15" bash profiles/phase_variants.sh $O phase && mv $O/phase.log $O/phase_c2.log \
 && PHASE_ARGS="c3 0" bash profiles/phase_variants.sh $O phase && mv $O/phase.log $O/phase_c3.log
