#!/bin/bash
# Round 4 run 36 (via gpurun): photon pass slots per photon (option 116: 8 / 16 (default) / 32 / 64, and
# the two-trace form) -- per-pass timings at C2 (bench diag pass), one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run36}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --steps 4 --warmup 1 --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'photon', round(d.get('photon_pass_ms',0),3), 'build', round(d.get('bvh_build_ms',0),3))"
}
for c in 0 8 16 32 64; do run slots$c --photon-single $c; done
run slots16b --photon-single 16
