#!/bin/bash
# r2: the tile kernel built with -fno-slp-vectorize (no packed-f32 SLP: fewer v_mov shuffles, 70 VGPRs):
# production parity tests, then C2 (16 iterations) at occupancy 6, 7 and 8, and C3 (1 iteration) at 6/7
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-occ_noslp}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for occ in 6 7 8; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --occupancy $occ --json-out $O/c2_occ$occ.json > $O/c2_occ$occ.log 2>&1 || { tail -n 20 $O/c2_occ$occ.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c2_occ$occ.json'));print('c2 occ $occ', round(d['value']), round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
done
for occ in 6 7; do
  timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --occupancy $occ --json-out $O/c3_occ$occ.json > $O/c3_occ$occ.log 2>&1 || { tail -n 20 $O/c3_occ$occ.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c3_occ$occ.json'));print('c3 occ $occ', round(d['value']), round(d['gather_kernel_ms'],1))"
done
