#!/bin/bash
# r2: exact-stage accumulation threshold BRE_RMW_MAX_RUNS (batches with more runs use LDS atomics):
# 0 (always atomics), 4, 8 (production), 16, 64 (never atomics)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-rmw_sweep}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
c2() { n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1))"
}
c3() { n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
P=beam-radiance-estimate-pbrt_amd/libbre.so
c2 prod $P && c2 rmw0 $V/libbre_rmw0.so && c2 rmw4 $V/libbre_rmw4.so && c2 rmw16 $V/libbre_rmw16.so && c2 rmw64 $V/libbre_rmw64.so \
 && c3 prod $P && c3 rmw4 $V/libbre_rmw4.so && c3 rmw16 $V/libbre_rmw16.so && c3 rmw64 $V/libbre_rmw64.so
