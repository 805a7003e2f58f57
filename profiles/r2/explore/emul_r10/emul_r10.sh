#!/bin/bash
# r2: packet-shard emulation (C2, N = 8, ranks 0 / 5 / 7; N = 2 rank 0) with the rank-accumulation kernel
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-emul_r10}; mkdir -p $O
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],2))"
}
c2 n1 && c2 r0of8 --emulate-shard 0/8 && c2 r5of8 --emulate-shard 5/8 && c2 r7of8 --emulate-shard 7/8 && c2 r0of2 --emulate-shard 0/2
