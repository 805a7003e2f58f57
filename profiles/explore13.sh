#!/bin/bash
# r2: occupancy / node-visit reload sweep of the RMW build, C2 4 iterations / C3 1
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore13}; mkdir -p $O
run() { # name, extra args...
  n=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-diag --steps 4 --warmup 1 --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || return 1
  timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --no-diag --steps 1 --warmup 0 --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || return 1
}
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run occ6b --occupancy 6 && run occ5 --occupancy 5 && run occ4 --occupancy 4 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1))"; done
