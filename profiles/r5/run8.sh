#!/bin/bash
# Round 5 run 8 (via gpurun): the serial work-root selection in one wave on cached nodes (k_roots):
# split / root-shard tests, per-segment sums bit for bit against the previous k_roots (variant base),
# C2 at N = 1 and an emulated rank of 8 (A/B/A/B), and a kernel trace of the default build for k_roots.
set -o pipefail
OUT=${1:-gpurun_out/r5/run8}
mkdir -p "$OUT"
export TMPDIR=/tmp
AB_TESTS="tests/test_split_gpu.py tests/test_root_shards_gpu.py tests/test_shard_gpu.py" \
  bash profiles/r5/ab.sh "$OUT" base || exit 1
run() { # name lib args...
  n=$1; lib=$2; shift 2
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), 'over', round(d['ms_per_step']-d['gather_kernel_ms'],2), 'build', round(d.get('bvh_build_ms',0),3))"
}
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
for r in a b; do
  run e8_def_$r beam-radiance-estimate-pbrt_amd/libbre.so --emulate-shard 0/8
  run e8_base_$r $V/libbre_base.so --emulate-shard 0/8
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu --no-diag --no-pmc --no-legs > "$OUT/trace.log" 2>&1 || { tail -n 20 "$OUT/trace.log"; exit 1; }
grep -i "k_roots\|k_refit\|k_pack" "$OUT/trace/run_kernel_stats.csv" | cut -d, -f1-4
