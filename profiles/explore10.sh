#!/bin/bash
# r2: ablations of the production gather (BRE_ABLATE 1 plain LDS stores instead of atomics, 2 no exact
# stage, 3 no prefilter scan), C2 4 iterations / C3 1 iteration, timing only (results are wrong)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore10}; mkdir -p $O
run() { # name, extra args...
  n=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-diag --steps 4 --warmup 1 --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || return 1
  timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --no-diag --steps 1 --warmup 0 --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || return 1
}
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run base && BRE_LIBRARY=$V/libbre_abl1.so run abl1 && BRE_LIBRARY=$V/libbre_abl2.so run abl2 && BRE_LIBRARY=$V/libbre_abl3.so run abl3 && run occ8 --occupancy 8 && run occ6 --occupancy 6 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1))"; done
