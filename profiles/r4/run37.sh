#!/bin/bash
# Round 4 run 37 (via gpurun): the photon pass with up to 64 slots per photon (2.5 GB scratch) --
# photon-form bit identity, photon / camera parity, C2 with per-pass timings, C3.
set -o pipefail
OUT=${1:-gpurun_out/r4/run37}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_photon_forms_gpu.py tests/test_photon_gpu.py tests/test_camera_gpu.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), 'photon', round(d.get('photon_pass_ms',0),3), 'build', round(d.get('bvh_build_ms',0),3))"
}
run n1
run r0of8 --emulate-shard 0/8
run c3 --workload c3 --steps 1 --warmup 1
