#!/bin/bash
# Round 3b run 2 (via gpurun): phase split of the run-1 kernel (C2 iterations 0 / 8 / 15, C3 0) and
# knob re-sweeps on it: transposed-scan threshold (4, 6, 8), RMW rounds (4, 8, 16), the node-reload
# build at occupancy 7.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run2}
mkdir -p "$OUT"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
BRE_LIBRARY=$V/libbre_phase.so timeout -k 10 200 python -u profiles/phase_timing.py c2 0 8 15 > "$OUT/phase_c2.log" 2>&1 \
    || { tail -n 20 "$OUT/phase_c2.log"; exit 1; }
BRE_LIBRARY=$V/libbre_phase.so timeout -k 10 200 python -u profiles/phase_timing.py c3 0 > "$OUT/phase_c3.log" 2>&1 \
    || { tail -n 20 "$OUT/phase_c3.log"; exit 1; }
grep iteration "$OUT"/phase_*.log
run() { # name env-or-empty args...
  n=$1; lib=$2; shift 2
  if [ -n "$lib" ]; then export BRE_LIBRARY=$V/libbre_$lib.so; else unset BRE_LIBRARY; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
run base ""
run tscan4 "" --tscan 4
run tscan8 "" --tscan 8
run rmw4 rmw4
run rmw16 rmw16
run reload7 reload --occupancy 7
run base2 ""
