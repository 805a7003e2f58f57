#!/bin/bash
# Round 3b run 10 (via gpurun): exact stage's square roots without the small-input scaling
# (sqrt_cr_noscale, default) -- per-segment sums and counts bit for bit against the sqrtf build
# (C2 iterations 0 and 8, C3), the production parity tests, then C2 / C3 A/B benches.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run10}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
for wl in c2 c3; do
  timeout -k 10 200 python -u profiles/r3b/bitcmp.py dump "$OUT/new_$wl.npz" $wl > "$OUT/dump_new_$wl.log" 2>&1 \
      || { tail -n 20 "$OUT/dump_new_$wl.log"; exit 1; }
  BRE_LIBRARY=$V/libbre_sqrt0.so timeout -k 10 200 python -u profiles/r3b/bitcmp.py dump "$OUT/old_$wl.npz" $wl \
      > "$OUT/dump_old_$wl.log" 2>&1 || { tail -n 20 "$OUT/dump_old_$wl.log"; exit 1; }
  python3 profiles/r3b/bitcmp.py cmp "$OUT/new_$wl.npz" "$OUT/old_$wl.npz"
done
rm -f "$OUT"/*.npz
T="tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { tail -n 30 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name lib args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run new ""
run old sqrt0
run new2 ""
run old2 sqrt0
run c3_new "" --workload c3 --steps 1 --warmup 0
run c3_old sqrt0 --workload c3 --steps 1 --warmup 0
