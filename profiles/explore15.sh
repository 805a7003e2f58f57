#!/bin/bash
# r2: exact-stage accumulation hybrid (RMW up to T runs per batch, LDS atomics beyond): C2 16 it., C3 1
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore15}; mkdir -p $O
run() { # name, extra args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || return 1
  timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --no-diag --steps 1 --warmup 0 --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || return 1
}
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run t4 && BRE_LIBRARY=$V/libbre_rmw2.so run t2 && BRE_LIBRARY=$V/libbre_rmw8.so run t8 && BRE_LIBRARY=$V/libbre_rmw64.so run t64 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), [round(x) for x in d['gather_ms_per_step']])"; done
