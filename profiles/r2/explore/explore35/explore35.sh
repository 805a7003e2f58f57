#!/bin/bash
# r2: S = 512 work roots under the LPT map (kMaxSplit 512), N=1 and an emulated 1/8 packet shard
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore35}; mkdir -p $O
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'gather', round(d['gather_kernel_ms'],1))"
}
c3() { n=$1; shift
  timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
c2 s256 && c2 s512 --split 512 && c2 p0of8s256 --emulate-shard 0/8 && c2 p0of8s512 --emulate-shard 0/8 --split 512 \
 && c3 s256 && c3 s512 --split 512
