#!/bin/bash
# r2: parameter re-sweep on the final kernel: work roots S (64/128/256), tile leaf 32, RMW run cap 4/16
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore26}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
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
c2 s64 $P && c2 s128 $P --split 128 && c2 s256 $P --split 256 && c2 leaf32 $P --tile-leaf 32 \
 && c2 rmw4 $V/libbre_rmw4.so && c2 rmw16 $V/libbre_rmw16.so \
 && c3 s64 $P && c3 s128 $P --split 128 && c3 s256 $P --split 256 && c3 rmw16 $V/libbre_rmw16.so
