#!/bin/bash
# r2: single-compare scan (thr * |thr| carries the lane-off / rejected-beam switches), T and occupancy
# on-lanes * 8 < kept beams * T.  Production parity tests, then C2 (16 it.) and C3 (1 it.) over T.
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore20}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
c3() {
  n=$1; shift
  timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
c2 t6 --tscan 6 && c2 t8 --tscan 8 && c2 t4 --tscan 4 && c2 t6o6 --tscan 6 --occupancy 6 \
 && c3 t6 --tscan 6 && c3 t8 --tscan 8 && c3 t6o6 --tscan 6 --occupancy 6
