#!/bin/bash
# Round 6 check 4 (via gpurun): the tile-kernel timing events, the pipeline / film tests, the default
# bench line (C3 / C4 / C5 legs, CPU leg, PMC roofline), then the multi-rank rehearsal.
set -o pipefail
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py \
    tests/test_film_determinism_gpu.py tests/test_pass_stream_gpu.py tests/test_bench_cli.py > "$OUT/pytest.log" 2>&1 \
    || { tail -n 40 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
timeout -k 10 600 python -u bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || { tail -n 30 "$OUT/bench.log"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "gather", round(d["gather_kernel_ms"], 3),
      "gap", round(d["ms_per_step"] - d["gather_kernel_ms"], 3), "it0", round(d["gather_ms_per_step"][0], 1),
      "it15", round(d["gather_ms_per_step"][15], 1), "digest", d["film_digest"]["sha256"])
r = d["roofline"]
print("roofline", r["bound"], round(r["frac"], 4), "launch_ms", round(r["launch_ms"], 1), "pmc_ms", r.get("pmc_launch_ms"),
      "td", r.get("issue", {}).get("td_busy_frac"), "vmem", r.get("issue", {}).get("SQ_INSTS_VMEM_RD"))
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
for k, v in d.get("config_legs", {}).items():
    print(k, {x: v.get(x) for x in ("iteration", "ranks_live", "gather_ms", "gather_estimates_per_s", "iteration_ms")},
          (v.get("film_digest") or {}).get("sha256"), v.get("error"))
print("late", d.get("counters_last_iteration", {}).get("gather_ms"), d.get("counters_last_iteration", {}).get("prefilter_tests_per_queued_pair"))
PY
bash profiles/r6/rehearse.sh "$OUT/rehearse"
