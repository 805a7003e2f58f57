#!/bin/bash
# r2: tile-kernel block mapping (XCD-aware subtrees vs rotated) and split, C2 4 iterations / C3 1
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore8}; mkdir -p $O
run() { # name, extra args...
  n=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --no-diag --steps 4 --warmup 1 --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || return 1
  timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --no-diag --steps 1 --warmup 0 --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || return 1
}
run map1s64 --block-map 1 --split 64 && run map2s16 --block-map 2 --split 16 && run map2s32 --block-map 2 --split 32 && run map1s32b --block-map 1 --split 32 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1))"; done
