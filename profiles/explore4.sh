#!/bin/bash
# r2: production-path parity, then C2 (4 iterations) / C3 (1 iteration) for: default build,
# scan mode 2, scan mode 2 with explicitly pipelined scalar loads (variant library).
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore4}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
run() { # name, extra args...
  n=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu --no-pmc --steps 4 --warmup 1 --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || return 1
  timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-pmc --steps 1 --warmup 0 --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || return 1
}
run m0 && run m2 --scan-mode 2 && BRE_LIBRARY=beam-radiance-estimate-pbrt_amd/csrc/build/variants/libbre_asm.so run asm --scan-mode 2 || exit 1
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', round(d['value']), round(d['gather_kernel_ms'],1), d.get('contributions_per_estimate'))"; done
