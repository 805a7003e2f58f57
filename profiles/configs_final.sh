#!/bin/bash
# r2 final kernel: C3 (1 iteration), C4 (N=1, 1 iteration) and the full C5 render (10 passes) at N=1
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-configs_final}; mkdir -p $O
timeout -k 10 200 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3.json > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --progress --json-out $O/c4.json > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
timeout -k 10 600 python -u bench.py --workload c5 --steps 10 --warmup 0 --no-cpu --no-pmc --no-diag --progress --json-out $O/c5.json > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
for f in c3 c4 c5; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', round(d['value']), round(d['ms_per_step']), [round(x) for x in d['gather_ms_per_step']])"; done
