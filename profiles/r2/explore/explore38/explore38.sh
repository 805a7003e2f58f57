#!/bin/bash
# r2: lane o / tmax / 1/d kept in registers through the traversal (BRE_NODE_RELOAD 0) at occupancy 6/7
# vs re-read from the SegRec at each node visit (production, occupancy 7)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore38}; mkdir -p $O
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
c2 prod $P && c2 nr0o6 $V/libbre_nr0.so --occupancy 6 && c2 nr0o7 $V/libbre_nr0.so --occupancy 7 \
 && c3 prod $P && c3 nr0o6 $V/libbre_nr0.so --occupancy 6
