#!/bin/bash
# r2: C2 16 iterations, occupancy 6 vs 7 (per-iteration gather times)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore14}; mkdir -p $O
for o in 6 7; do
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --occupancy $o --json-out $O/c2_occ$o.json > $O/c2_occ$o.log 2>&1 || exit 1
done
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), [round(x) for x in d['gather_ms_per_step']])"; done
