#!/bin/bash
# Round 4 run 15 (via gpurun): leaf-tile size sweep (BRE_OPT_TILE_LEAF 64 / 48 / 32 / 16) on C2,
# per-iteration gather times, and the scan shape at iterations 0 / 8 / 15 for 64 and 32.
set -o pipefail
OUT=${1:-gpurun_out/r4/run15}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
for l in 64 48 32 16; do run c2_leaf$l $NEW --tile-leaf $l; done
run c3_leaf64 $NEW --workload c3 --steps 1 --warmup 1
run c3_leaf32 $NEW --workload c3 --steps 1 --warmup 1 --tile-leaf 32
for l in 64 32; do
  BRE_LIBRARY=$V/libbre_scan.so timeout -k 10 200 python -u profiles/scan_stats.py c2 0 8 15 opt:10=$l > "$OUT/scan_leaf$l.log" 2>&1 \
      || { echo "scan failed"; tail -n 20 "$OUT/scan_leaf$l.log"; exit 1; }
  echo "== leaf $l"; grep iteration "$OUT/scan_leaf$l.log"
done
