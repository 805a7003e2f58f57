#!/bin/bash
# r2: work roots S and occupancy re-checked under the LPT block map (C2 16 iterations, C3 1)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore33}; mkdir -p $O
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'gather', round(d['gather_kernel_ms'],1))"
}
c3() { n=$1; shift
  timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
c2 s256 && c2 s128 --split 128 && c2 s64 --split 64 && c2 s256o6 --occupancy 6 && c2 s256t4 --tscan 4 \
 && c3 s256 && c3 s128 --split 128 && c3 s256o6 --occupancy 6
