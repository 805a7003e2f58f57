#!/bin/bash
# Round 4 run 6 (via gpurun): what the deterministic accumulation costs -- film compose vs float
# atomics (option 114), read-modify-write rounds to 64 vs 8 + LDS atomics (BRE_RMW_ROUNDS), against
# the round-3 library, C2 and C3, one box (timing only).
set -o pipefail
OUT=${1:-gpurun_out/r4/run6}
mkdir -p "$OUT"
export TMPDIR=/tmp
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
run c2_film0 $NEW --film-compose 0
run c2_rr8 $V/libbre_rr8.so
run c2_rr8_film0 $V/libbre_rr8.so --film-compose 0
run c2_r3 $V/libbre_r3.so
run c2_nopipe $NEW --pipeline 0
run c3_new $NEW $C3
run c3_film0 $NEW $C3 --film-compose 0
run c3_rr8 $V/libbre_rr8.so $C3
run c3_r3 $V/libbre_r3.so $C3
run c2_new2 $NEW
