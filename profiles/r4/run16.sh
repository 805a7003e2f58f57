#!/bin/bash
# Round 4 run 16 (via gpurun): the 4-wide walk of the tile tree (BRE_TREE4, Node4) -- the whole GPU
# suite, then C2 / C3 against the binary walk (variant bin) on one box, and the phase split of both at
# C2 iterations 0 / 8 / 15.
set -o pipefail
OUT=${1:-gpurun_out/r4/run16}
mkdir -p "$OUT"
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d.get('gather_ms_per_step',[])])"
}
C3="--workload c3 --steps 1 --warmup 1"
NEW=beam-radiance-estimate-pbrt_amd/libbre.so
run c2_t4 $NEW
run c2_bin $V/libbre_bin.so
run c3_t4 $NEW $C3
run c3_bin $V/libbre_bin.so $C3
run c2_t4b $NEW
for n in phase binphase; do
  BRE_LIBRARY=$V/libbre_$n.so timeout -k 10 200 python -u profiles/phase_timing.py c2 0 8 15 > "$OUT/$n.log" 2>&1 \
      || { echo "phase failed"; tail -n 20 "$OUT/$n.log"; exit 1; }
  echo "== $n"; grep iteration "$OUT/$n.log"
done
