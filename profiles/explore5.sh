#!/bin/bash
# r2: packet box reject -- production-path parity, C2 (4 iterations) / C3 (1 iteration) with counters
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore5}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --steps 4 --warmup 1 --json-out $O/c2.json > $O/c2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --steps 1 --warmup 0 --json-out $O/c3.json > $O/c3.log 2>&1 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1), d.get('contributions_per_estimate'), d.get('bundle_keep_frac'), d.get('exact_batches_per_wave'))"; done
