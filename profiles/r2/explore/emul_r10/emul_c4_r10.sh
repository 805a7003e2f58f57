#!/bin/bash
# r2: C4 packet-shard emulation (N = 8 ranks 0 / 5) with the rank-accumulation kernel
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-emul_r10}; mkdir -p $O
c4() { n=$1; shift
  timeout -k 10 300 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --progress --json-out $O/c4_$n.json "$@" > $O/c4_$n.log 2>&1 || { tail -n 20 $O/c4_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c4_$n.json'));print('c4 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1))"
}
c4 r0of8 --emulate-shard 0/8 && c4 r5of8 --emulate-shard 5/8
