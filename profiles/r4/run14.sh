#!/bin/bash
# Round 4 run 14 (via gpurun): the tile line reject with the region-wide threshold only (the
# packet-local threshold removed after run 13), option / parity / determinism tests; then where the
# remaining cost against round 3 sits, on one box: the reject compiled out (nt), round 3's
# accumulation (r3acc: ds_add ranks, float atomics past 8 rounds), both (ntr3), the ds_or ranks
# without the order check (rk2), the round-3 library; C2 and C3.
set -o pipefail
OUT=${1:-gpurun_out/r4/run14}
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
for w in c2 c3; do
  A=""; [ $w = c3 ] && A=$C3
  run ${w}_new $NEW $A
  run ${w}_off $NEW $A --tile-axis 0
  run ${w}_nt $V/libbre_nt.so $A
  run ${w}_r3acc $V/libbre_r3acc.so $A
  run ${w}_ntr3 $V/libbre_ntr3.so $A
  run ${w}_rk2 $V/libbre_rk2.so $A
  run ${w}_r3 $V/libbre_r3.so $A
  run ${w}_new2 $NEW $A
done
