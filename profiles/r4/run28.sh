#!/bin/bash
# Round 4 run 28 (via gpurun): the single-trace photon pass (option 116) -- forms bit-identical, photon /
# camera / C2 parity tests, then C2 with per-pass timings (single vs two traces), N = 1 and rank 0 of 8.
set -o pipefail
OUT=${1:-gpurun_out/r4/run28}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_photon_forms_gpu.py tests/test_photon_gpu.py tests/test_camera_gpu.py tests/test_c2_production.py \
    tests/test_film_determinism_gpu.py tests/test_c3_c5_gpu.py > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), 'photon', round(d.get('photon_pass_ms',0),3), 'build', round(d.get('bvh_build_ms',0),3), 'camera', round(d.get('camera_pass_ms',0),3))"
}
run n1
run r0of8 --emulate-shard 0/8
run c3 --workload c3 --steps 1 --warmup 1
run n1_two --photon-single 0
