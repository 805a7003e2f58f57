#!/bin/bash
# r2: scan shape and phase split of the final kernel (LPT map)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore37}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
BRE_LIBRARY=$V/libbre_scan.so timeout -k 10 200 python -u profiles/scan_stats.py c2 0 8 15 > $O/scan_c2.log 2>&1 || { tail $O/scan_c2.log; exit 1; }
BRE_LIBRARY=$V/libbre_scan.so timeout -k 10 200 python -u profiles/scan_stats.py c3 0 > $O/scan_c3.log 2>&1 || { tail $O/scan_c3.log; exit 1; }
cat $O/scan_c2.log $O/scan_c3.log | grep iteration
PHASE_ARGS="c2 0 8 15" bash profiles/phase_variants.sh $O phase && mv $O/phase.log $O/phase_c2.log \
 && PHASE_ARGS="c3 0" bash profiles/phase_variants.sh $O phase && mv $O/phase.log $O/phase_c3.log
