#!/bin/bash
# r2: the full C5 render at N=1 -- 10 progressive passes, 1024^2, grid smoke, 50M photons per pass
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-c5full}; mkdir -p $O
timeout -k 10 1080 python -u bench.py --workload c5 --no-cpu --no-pmc --no-diag --steps 10 --warmup 0 --progress \
    --json-out $O/c5.json 2>&1 | tee $O/c5.log || exit 1
python3 -c "import json;d=json.load(open('$O/c5.json'));print('c5', round(d['value']), d['ms_per_step'], [round(x) for x in d['gather_ms_per_step']])"
