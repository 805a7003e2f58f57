#!/bin/bash
# r2: with the rank accumulation, re-check the node-reload build at occupancy 7 and the work-root
# count S (--split 64 / 128; 256 is the maximum) against production (S 256, registers, occupancy 6)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-occ_split_r10}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
P=beam-radiance-estimate-pbrt_amd/libbre.so
c2() { n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1))"
}
c2 prod $P && c2 nr1o7 $V/libbre_nr1.so --occupancy 7 && c2 s128 $P --split 128 && c2 s64 $P --split 64
