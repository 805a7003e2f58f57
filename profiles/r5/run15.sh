#!/bin/bash
# Round 5 run 15 / 16 (via gpurun): build changes (15: hash-keyed 32-bit centroid sort; 16: wave-run photon slot copy, k_pack without centroid reads; 17: leaf boxes one wave per leaf) --
# build / group-box tests, per-segment sums bit for bit against HEAD's full native tree (variant
# base), C2 N = 1 and emulated rank of 8 timing, A/B/A/B.
set -o pipefail
OUT=${1:-gpurun_out/r5/run15}
mkdir -p "$OUT"
export TMPDIR=/tmp
AB_TESTS="tests/test_chunk_gpu.py tests/test_shard_gpu.py tests/test_split_gpu.py" bash profiles/r5/ab.sh "$OUT" base || exit 1
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
