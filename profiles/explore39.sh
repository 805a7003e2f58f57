#!/bin/bash
# r2: four kept beams per beam-major scan step (BRE_SCAN_BEAMS 4, queue 320 slots) vs two
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore39}; mkdir -p $O
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
BRE_LIBRARY=$V/libbre_b4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "production or prefilter or transposed" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1))"
}
c3() { n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
P=beam-radiance-estimate-pbrt_amd/libbre.so
c2 b2 $P && c2 b4 $V/libbre_b4.so && c2 b2b $P && c2 b4b $V/libbre_b4.so && c3 b2 $P && c3 b4 $V/libbre_b4.so
