#!/bin/bash
# Round 4 run 17 (via gpurun): the shift-form lane-order check (in-tree), then the exact stage's segment
# values by ds_bpermute (shfl1: o, tmax, 1/d, au; shfl3: all of them, no SegRec load) against it, C2 / C3.
set -o pipefail
OUT=${1:-gpurun_out/r4/run17}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prefilter_options_gpu.py tests/test_gpu_parity.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
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
for w in c2 c3; do
  A=""; [ $w = c3 ] && A=$C3
  run ${w}_new $NEW $A
  run ${w}_shfl1 $V/libbre_shfl1.so $A
  run ${w}_shfl3 $V/libbre_shfl3.so $A
  run ${w}_bin $V/libbre_bin.so $A
done
