#!/bin/bash
# Round 4 run 13 (via gpurun): the tile line reject with the packet-local threshold (option 112 = 1,
# default), the region-wide threshold only (2), off (0) -- option / parity tests, C2 / C3 timing against
# the queue count compiled out (nq), round 3's accumulation without the reject (r3like) and the round-3
# library; then the scan shape of C2 iterations 0 / 8 / 15 in the three modes.
set -o pipefail
OUT=${1:-gpurun_out/r4/run13}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
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
run c2_local $NEW
run c2_region $NEW --tile-axis 2
run c2_off $NEW --tile-axis 0
run c2_nq $V/libbre_nq.so
run c2_r3like $V/libbre_r3like.so
run c2_r3 $V/libbre_r3.so
run c3_local $NEW $C3
run c3_region $NEW $C3 --tile-axis 2
run c3_off $NEW $C3 --tile-axis 0
run c3_r3 $V/libbre_r3.so $C3
run c2_local2 $NEW
run c2_ts4 $NEW --tscan 4
run c2_ts8 $NEW --tscan 8
run c2_ts12 $NEW --tscan 12
for t in 1 2 0; do
  BRE_LIBRARY=$V/libbre_scan.so timeout -k 10 200 python -u profiles/scan_stats.py c2 0 8 15 opt:112=$t > "$OUT/scan_tax$t.log" 2>&1 \
      || { echo "scan failed"; tail -n 20 "$OUT/scan_tax$t.log"; exit 1; }
  echo "== tax $t"; grep iteration "$OUT/scan_tax$t.log"
done
