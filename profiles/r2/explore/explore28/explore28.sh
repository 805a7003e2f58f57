#!/bin/bash
# r2: strong-scaling emulation on one GPU (block: tiles per side of the blocks dealt to the ranks): rank R's share of an N-GPU run (its 16x16 tiles, all the
# photons, its own BVH), C2 16 iterations; efficiency ~ T(N=1) / (N * max_R T(R of N))
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore28}; mkdir -p $O
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'gather', round(d['gather_kernel_ms'],1), 'seg/step', round(d['estimates_per_step_per_gpu']))"
}
c2 n1 && c2 r0of8 --emulate-shard 0/8 && c2 r5of8 --emulate-shard 5/8 \
 && c2 r0of8b2 --emulate-shard 0/8 --shard-block 2 && c2 r5of8b2 --emulate-shard 5/8 --shard-block 2 \
 && c2 r0of8b4 --emulate-shard 0/8 --shard-block 4 && c2 r5of8b4 --emulate-shard 5/8 --shard-block 4 \
 && c2 r3of8b4 --emulate-shard 3/8 --shard-block 4 && c2 r0of2 --emulate-shard 0/2 && c2 r0of2b4 --emulate-shard 0/2 --shard-block 4
