#!/bin/bash
# r2: packet-plane SegRec layout (plane k of a packet contiguous) vs one 64-B record per segment
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore24}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
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
c2 plane $P && c2 aos $V/libbre_aos.so && c2 plane_b $P && c2 aos_b $V/libbre_aos.so \
 && c3 plane $P && c3 aos $V/libbre_aos.so
