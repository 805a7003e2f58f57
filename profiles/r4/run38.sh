#!/bin/bash
# Round 4 run 38 (via gpurun): work-root shards (--shard-mode roots, BRE_OPT_SHARD_MODE 2) -- the shards
# sum to one shard (test), then emulated ranks of 2 / 4 / 8 against packet shards, C2, one box.
set -o pipefail
OUT=${1:-gpurun_out/r4/run38}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_root_shards_gpu.py tests/test_pipeline_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), [round(x,1) for x in d.get('gather_ms_per_step',[])][:4])"
}
run n1
for m in packets roots; do
  run ${m}_0of8 --emulate-shard 0/8 --shard-mode $m
  run ${m}_7of8 --emulate-shard 7/8 --shard-mode $m
  run ${m}_0of4 --emulate-shard 0/4 --shard-mode $m
  run ${m}_0of2 --emulate-shard 0/2 --shard-mode $m
done
run roots_3of8 --emulate-shard 3/8 --shard-mode roots
run c4_roots_0of8 --workload c4 --steps 1 --warmup 0 --emulate-shard 0/8 --shard-mode roots
