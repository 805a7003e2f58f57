#!/bin/bash
# r2: C4 (2048^2 fog, 20M photons, 1 iteration) strong-scaling emulation: ranks 0 and 5 of 8 and rank 0
# of 2, packet shards (N=1 reference: profiles/r2/configs/final_c4.json, 101.0 s)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore36}; mkdir -p $O
c4() { n=$1; shift
  timeout -k 10 400 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c4_$n.json "$@" > $O/c4_$n.log 2>&1 || { tail -n 20 $O/c4_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c4_$n.json'));print('c4 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'seg/step', round(d['estimates_per_step_per_gpu']))"
}
c4 r0of8 --emulate-shard 0/8 && c4 r5of8 --emulate-shard 5/8 && c4 r0of2 --emulate-shard 0/2
