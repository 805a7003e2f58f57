#!/bin/bash
# r2: C4 (2048^2 fog, 20M photons, 1 iteration) and C5 (1024^2 smoke, 50M photons, 2 of its 10
# iterations) at N=1, no CPU leg / PMC / counter pass (each iteration is a long kernel)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-configs}; mkdir -p $O
timeout -k 10 420 python -u bench.py --workload c4 --no-cpu --no-pmc --no-diag --steps 1 --warmup 0 --json-out $O/c4.json > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
timeout -k 10 540 python -u bench.py --workload c5 --no-cpu --no-pmc --no-diag --steps 2 --warmup 0 --json-out $O/c5.json > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
for f in $O/c4.json $O/c5.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), d['ms_per_step'], [round(x) for x in d['gather_ms_per_step']], d.get('beams_per_iteration'))"; done
