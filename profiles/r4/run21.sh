#!/bin/bash
# Round 4 run 21 (via gpurun): where an emulated 1/8 rank's C2 iteration goes -- with the two-context
# pipeline (default) and without it (--pipeline 0: passes and gather serialised), N = 1 and rank 0 of 8.
set -o pipefail
OUT=${1:-gpurun_out/r4/run21}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), 'photon', round(d.get('photon_pass_ms',0),2), 'build', round(d.get('bvh_build_ms',0),2), 'camera', round(d.get('camera_pass_ms',0),2))"
}
run n1_p1
run n1_p0 --pipeline 0
run r0of8_p1 --emulate-shard 0/8
run r0of8_p0 --emulate-shard 0/8 --pipeline 0
