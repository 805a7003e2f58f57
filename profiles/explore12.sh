#!/bin/bash
# r2: phase split of the current gather (C2 iterations 0/8, C3 iteration 0) + SQ counters (C3 pass)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore12}; mkdir -p $O
export TMPDIR=/tmp
PHASE_ARGS="c3 0" timeout -k 10 300 bash profiles/phase_variants.sh $O/phase_c3 phase || exit 1
PHASE_ARGS="c2 0 8" timeout -k 10 300 bash profiles/phase_variants.sh $O/phase_c2 phase || exit 1
timeout -k 10 600 python -u bench.py --no-cpu --steps 4 --warmup 1 --json-out $O/c2.json > $O/c2.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --workload c3 --no-cpu --steps 1 --warmup 0 --json-out $O/c3.json > $O/c3.log 2>&1 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1), json.dumps(d['roofline'].get('issue')))"; done
