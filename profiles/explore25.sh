#!/bin/bash
# r2: per-run beam-line broadcast in the exact stage (BRE_RUN_BCAST runs at most) vs per-lane loads
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore25}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
c3() {
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
P=beam-radiance-estimate-pbrt_amd/libbre.so
c2 bc16 $P && c2 bc0 $V/libbre_bc0.so && c2 bc8 $V/libbre_bc8.so && c2 bc64 $V/libbre_bc64.so && c2 bc16o6 $P --occupancy 6 \
 && c3 bc16 $P && c3 bc0 $V/libbre_bc0.so && c3 bc64 $V/libbre_bc64.so
