#!/bin/bash
# Round 3b run 3 (via gpurun): separable packet line reject (default build) -- production parity
# tests; the exact stage taking the segment's values from its lane by ds_bpermute (variant shfl: o,
# tmax, 1/d, au, has_inf; shfl2: the box-test values only) -- its parity tests; C2 benches of the
# default, shfl, shfl2 and no-box-reject builds on one box; C3 default vs shfl.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run3}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
T="tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { tail -n 30 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
BRE_LIBRARY=$V/libbre_shfl.so timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_shfl.log" 2>&1 || { tail -n 30 "$OUT/pytest_shfl.log"; exit 1; }
tail -n 1 "$OUT/pytest_shfl.log"
run() { # name lib args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]], 'keep', round(d.get('bundle_keep_frac',0),3))"
}
run base ""
run shfl shfl
run shfl2 shfl2
run nobox nobox
run base2 ""
run c3 "" --workload c3 --steps 1 --warmup 0
run c3_shfl shfl --workload c3 --steps 1 --warmup 0
