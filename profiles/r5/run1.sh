#!/bin/bash
# Round 5 run 1 (via gpurun): the matrix-pipe prefilter scan (BRE_MFMA_SCAN, scan_group) -- parity /
# option / determinism tests, per-segment sums bit for bit against the VALU scan (variant valu) at C2
# iterations 0 / 8 / 15 and C3, then C2 / C3 timing of both on one box.
set -o pipefail
OUT=${1:-gpurun_out/r5/run1}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
for lib in mfma valu; do
  for w in c2 c3; do
    BRE_LIBRARY=$V/libbre_$lib.so timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_${lib}_$w.npz" $w \
        > "$OUT/bc_${lib}_$w.log" 2>&1 || { tail -n 20 "$OUT/bc_${lib}_$w.log"; exit 1; }
  done
done
for w in c2 c3; do python3 profiles/r5/bitcmp.py cmp "$OUT/bc_mfma_$w.npz" "$OUT/bc_valu_$w.npz"; done
rm -f "$OUT"/*.npz  # (too large to copy back)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 3 "$OUT/pytest.log"
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x,1) for x in d.get('gather_ms_per_step',[])])"
}
C3="--workload c3 --steps 1 --warmup 1"
run c2_mfma $V/libbre_mfma.so
run c2_valu $V/libbre_valu.so
run c3_mfma $V/libbre_mfma.so $C3
run c3_valu $V/libbre_valu.so $C3
run c2_mfma_b $V/libbre_mfma.so
run c2_valu_b $V/libbre_valu.so
