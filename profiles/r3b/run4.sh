#!/bin/bash
# Round 3b run 4 (via gpurun): exact stage through buffer descriptors (variant buf: SegRec planes and
# power by SGPR base + 32-bit lane offset) -- its parity tests; the price of the ordered rank
# accumulation (variant acc1: one racy RMW round, wrong sums, timing only); C2 and C3 benches.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run4}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
T="tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py"
BRE_LIBRARY=$V/libbre_buf.so timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_buf.log" 2>&1 || { tail -n 30 "$OUT/pytest_buf.log"; exit 1; }
tail -n 1 "$OUT/pytest_buf.log"
run() { # name lib args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run base ""
run buf buf
run acc1 acc1
run bufacc1 bufacc1
run base2 ""
run c3 "" --workload c3 --steps 1 --warmup 0
run c3_buf buf --workload c3 --steps 1 --warmup 0
run c3_acc1 acc1 --workload c3 --steps 1 --warmup 0
