#!/bin/bash
# r2: scan mode 2 (scalar-loaded scan records) vs mode 0 at C2 (4 iterations) and C3 (1 iteration)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore2}; mkdir -p $O
for m in 0 2; do
timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --steps 4 --warmup 1 --scan-mode $m --json-out $O/c2_scan$m.json > $O/c2_scan$m.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --steps 1 --warmup 0 --scan-mode 2 --json-out $O/c3_scan2.json > $O/c3_scan2.log 2>&1 && timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --steps 1 --warmup 0 --scan-mode 0 --json-out $O/c3_scan0.json > $O/c3_scan0.log 2>&1 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1), d.get('contributions_per_estimate'))"; done
