#!/bin/bash
# r2: transposed-scan threshold (--tscan; production 6) re-swept with the rank accumulation
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-tscan_r10}; mkdir -p $O
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1))"
}
c3() { n=$1; shift
  timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
c2 t6 && c2 t0 --tscan 0 && c2 t4 --tscan 4 && c2 t8 --tscan 8 && c2 t12 --tscan 12 && c3 t6 && c3 t4 --tscan 4 && c3 t8 --tscan 8
