#!/bin/bash
# Round 3b run 19 (via gpurun): the exact stage recomputes the segment's unit direction instead of
# loading SegRec plane 2 (seven vector loads per pair) -- parity tests, then C2 / C3 A/B against the
# loading build (variant au0).
set -o pipefail
OUT=${1:-gpurun_out/r3b/run19}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_radius_layout_gpu.py tests/test_gpu_parity.py tests/test_prefilter_options_gpu.py tests/test_c2_production.py \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
run() { # name lib args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run au ""
run au0 au0
C3="--workload c3 --steps 1 --warmup 0"
run c3_au "" $C3
run c3_au0 au0 $C3
run au_b ""
run au0_b au0
