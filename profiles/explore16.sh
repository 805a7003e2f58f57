#!/bin/bash
# r2: work roots per packet 64 / 128 / 256, C2 16 it., C3 1
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore16}; mkdir -p $O
run() { # name, extra args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || return 1
  timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --no-diag --steps 1 --warmup 0 --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || return 1
}
run s64 --split 64 && run s128 --split 128 && run s256 --split 256 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), [round(x) for x in d['gather_ms_per_step']])"; done
