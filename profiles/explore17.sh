#!/bin/bash
# r2: no-SLP build (-fno-slp-vectorize: no packed-f32 shuffles, 70-76 VGPRs) and the squared scan
# prefilter (BRE_SCAN_SQ, no v_sqrt per (lane, beam)).  Production parity tests on the production
# library, then C2 (16 iterations) and C3 (1 iteration) per variant and occupancy.
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore17}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { # name lib occ
  BRE_LIBRARY=$2 timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --occupancy $3 --json-out $O/c2_$1.json > $O/c2_$1.log 2>&1 || { tail -n 20 $O/c2_$1.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$1.json'));print('c2 $1', round(d['value']), round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
c3() {
  BRE_LIBRARY=$2 timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --occupancy $3 --json-out $O/c3_$1.json > $O/c3_$1.log 2>&1 || { tail -n 20 $O/c3_$1.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$1.json'));print('c3 $1', round(d['value']), round(d['gather_kernel_ms'],1))"
}
P=beam-radiance-estimate-pbrt_amd/libbre.so
c2 slp_nosq_6 $V/libbre_slp_nosq.so 6 && c2 noslp_nosq_6 $V/libbre_noslp_nosq.so 6 && c2 noslp_nosq_7 $V/libbre_noslp_nosq.so 7 \
 && c2 prod_6 $P 6 && c2 prod_7 $P 7 && c2 prod_8 $P 8 \
 && c3 slp_nosq_6 $V/libbre_slp_nosq.so 6 && c3 noslp_nosq_6 $V/libbre_noslp_nosq.so 6 && c3 prod_6 $P 6 && c3 prod_7 $P 7
