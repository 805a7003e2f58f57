#!/bin/bash
# r2 exploration: scan mode A/B at C2, C3 phase split and bench.
set -o pipefail
O=gpurun_out/explore1; mkdir -p $O
timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --steps 4 --warmup 1 --json-out $O/c2_scan0.json > $O/c2_scan0.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --steps 4 --warmup 1 --scan-mode 1 --json-out $O/c2_scan1.json > $O/c2_scan1.log 2>&1 || exit 1
PHASE_ARGS="c3 0" timeout -k 10 300 bash profiles/phase_variants.sh $O/phase_c3 phase || exit 1
PHASE_ARGS="c2 0 8" timeout -k 10 300 bash profiles/phase_variants.sh $O/phase_c2 phase || exit 1
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --steps 1 --warmup 0 --json-out $O/c3.json > $O/c3.log 2>&1 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1))"; done
