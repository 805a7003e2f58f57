#!/bin/bash
# Round 5 run 2 (via gpurun): the passes on a high-priority stream (option 117, PassStream in
# bre_api.hip) -- pipeline / determinism tests; the driver-shaped bench line with the new late-funnel
# counters and the C3 / C4 legs; C2 with the option off; an emulated rank of 8 both ways; the rocprofv3
# kernel trace of the pipelined render (k_photons / k_camera per dispatch).
set -o pipefail
OUT=${1:-gpurun_out/r5/run2}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_pipeline_gpu.py tests/test_film_determinism_gpu.py tests/test_boundary_gpu.py \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
    || { tail -n 30 "$OUT/bench.log"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2), "gather", round(d["gather_kernel_ms"], 2))
print("per step", [round(x, 1) for x in d["gather_ms_per_step"]])
c = d.get("counters_last_iteration", {})
print("late counters: iteration", c.get("iteration"), "gather_ms", c.get("gather_ms"), "tests/queued", c.get("prefilter_tests_per_queued_pair"))
print("cpu", {k: d["cpu_baseline"].get(k) for k in ("value", "cores", "value_1_thread")})
print("roofline", {k: d["roofline"].get(k) for k in ("bound", "achieved", "peak", "frac", "traffic")})
print("legs", json.dumps(d.get("config_legs"))[:1500])
PY
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2))"
}
run pp0 --steps 20 --warmup 5 --pass-priority 0
run pp1 --steps 20 --warmup 5
run e8_pp1 --steps 16 --emulate-shard 0/8
run e8_pp0 --steps 16 --emulate-shard 0/8 --pass-priority 0
bash profiles/run_profiles.sh "$OUT/prof" --steps 16 --warmup 1 --no-legs || { tail -n 20 "$OUT"/prof/bench_*.log; exit 1; }
python3 - "$OUT/prof/profile_summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if v.get("median_dispatch_ms") is not None:
        print(k, "calls", v.get("calls"), "avg_ms", round(v["avg_ns"] * 1e-6, 3), "median_ms", v["median_dispatch_ms"], "max", max(v["dispatch_ms"]))
PY
