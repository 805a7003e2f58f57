#!/bin/bash
# r2: exact-stage accumulation by per-segment rank (BRE_ACC_RANK 1) vs per-run RMW (production):
# bit identity of one C2 iteration, then C2 / C3 throughput
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-acc_rank}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
P=beam-radiance-estimate-pbrt_amd/libbre.so
H=profiles/r2/explore/acc_rank/ldhash.py
c2() { n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1))"
}
c3() { n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
BRE_LIBRARY=$P timeout -k 10 120 python -u $H c2 3 && BRE_LIBRARY=$V/libbre_rk8.so timeout -k 10 120 python -u $H c2 3 \
 && c2 prod $P && c2 rk8 $V/libbre_rk8.so && c2 rk4 $V/libbre_rk4.so && c2 rk16 $V/libbre_rk16.so \
 && c3 prod $P && c3 rk8 $V/libbre_rk8.so && c3 rk16 $V/libbre_rk16.so
