#!/bin/bash
# Round 4 run 9 (via gpurun): verified lane-order ranks (ds_or_rtn_b64 + one ballot check) -- tests,
# C2 / C3 timing (tile line reject on / off, 8 rounds + atomics variant, round 3), then the phase split
# and scan shape of C2 iterations 0 / 8 / 15 with the tile line reject on and off.
set -o pipefail
OUT=${1:-gpurun_out/r4/run9}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_prefilter_options_gpu.py tests/test_film_determinism_gpu.py \
    tests/test_c2_production.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 3 "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
C3="--workload c3 --steps 1 --warmup 1"
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
run c2_new $NEW
run c2_tax $NEW --tile-axis 1
run c2_rr8_tax $V/libbre_rr8.so --tile-axis 1
run c2_r3 $V/libbre_r3.so
run c3_new $NEW $C3
run c3_tax $NEW $C3 --tile-axis 1
run c3_r3 $V/libbre_r3.so $C3
for t in 0 1; do
  BRE_LIBRARY=$V/libbre_phase.so timeout -k 10 200 python -u profiles/phase_timing.py c2 0 8 15 opt:112=$t > "$OUT/phase_tax$t.log" 2>&1 \
      || { echo "phase failed"; tail -n 20 "$OUT/phase_tax$t.log"; exit 1; }
  BRE_LIBRARY=$V/libbre_scan.so timeout -k 10 200 python -u profiles/scan_stats.py c2 0 8 15 opt:112=$t > "$OUT/scan_tax$t.log" 2>&1 \
      || { echo "scan failed"; tail -n 20 "$OUT/scan_tax$t.log"; exit 1; }
  echo "== tax $t"; grep iteration "$OUT/phase_tax$t.log" "$OUT/scan_tax$t.log"
done
