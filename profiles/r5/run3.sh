#!/bin/bash
# Round 5 run 3 (via gpurun): tighter packet bundle line (BRE_BUNDLE_LINE: through the centres of the
# lanes' origin / end boxes) and tile axis (BRE_AXIS_BOX: through the centres of the beams' start / end
# boxes) -- per-segment sums bit for bit against the default build, then C2 (counters at iterations 0 and
# 15: kept fraction, tests per queued pair) and C3 timing of the four builds on one box.
set -o pipefail
OUT=${1:-gpurun_out/r5/run3}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
# the round's new GPU tests first: packet-class films (bit-identical N-shard films), work-root shard
# refusals / XCD map fallback / empty packet shard, the full-size C1 image against the oracle chain
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
    tests/test_shard_gpu.py tests/test_root_shards_gpu.py tests/test_pipeline_gpu.py \
    tests/test_film_determinism_gpu.py tests/test_pbrt_gpu.py tests/test_c2_production.py tests/test_gpu_parity.py \
    tests/test_prefilter_options_gpu.py > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
grep -E "^C1 full film" "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
DEF=beam-radiance-estimate-pbrt_amd/libbre.so
for lib in $DEF $V/libbre_blax.so; do
  n=$(basename $lib .so)
  BRE_LIBRARY=$lib timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_$n.npz" c2 > "$OUT/bc_$n.log" 2>&1 \
      || { tail -n 20 "$OUT/bc_$n.log"; exit 1; }
done
python3 profiles/r5/bitcmp.py cmp "$OUT/bc_libbre.npz" "$OUT/bc_libbre_blax.npz"
rm -f "$OUT"/*.npz
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); n = sys.argv[2]
c = d.get("counters_last_iteration") or {}
print(n, "value", round(d["value"]), "gather", round(d["gather_kernel_ms"], 1), "it0", round(d["gather_ms_per_step"][0], 1),
      "it15", round(d["gather_ms_per_step"][-1], 1) if len(d["gather_ms_per_step"]) > 15 else None,
      "keep", round(d.get("bundle_keep_frac", 0), 4), "t/q", round(d.get("prefilter_tests_per_queued_pair", 0), 2),
      "| late keep", round(c.get("bundle_keep_frac", 0), 4), "t/q", round(c.get("prefilter_tests_per_queued_pair", 0), 2),
      "leaf/wave", round(c.get("leaf_visits_per_wave", 0), 2))
PY
}
C3="--workload c3 --steps 1 --warmup 1"
for lib in $DEF $V/libbre_bl.so $V/libbre_ax.so $V/libbre_blax.so; do
  n=$(basename $lib .so)
  run c2_$n $lib
done
for lib in $DEF $V/libbre_blax.so; do
  n=$(basename $lib .so)
  run c3_$n $lib $C3
done
run c2_libbre_b $DEF
run c2_libbre_blax_b $V/libbre_blax.so
# the pipelined render after the scene-record upload is skipped when unchanged (kernel trace)
bash profiles/run_profiles.sh "$OUT/prof" --steps 16 --warmup 1 --no-legs || { tail -n 20 "$OUT"/prof/bench_*.log; exit 1; }
python3 - "$OUT/prof" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_trace.csv")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
g = [e for e in ev if "k_gather_tile" in e[2]]
gaps = [(g[i + 1][0] - g[i][1]) / 1e6 for i in range(len(g) - 1)]
print("gaps between gather kernels (ms):", [round(x, 2) for x in gaps])
ph = sorted((e[1] - e[0]) / 1e6 for e in ev if "k_photons<2>" in e[2])
print("k_photons<2> ms: median", round(ph[len(ph) // 2], 3), "max", round(ph[-1], 3))
cp = sorted((e[1] - e[0]) / 1e6 for e in ev if "copyBuffer" in e[2])
print("copyBuffer ms: max", round(cp[-1], 3), "n", len(cp))
PY
