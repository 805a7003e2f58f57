#!/bin/bash
# Round 3b run 9 (via gpurun): the multi-rank bench flow rehearsed on one GPU (2 packet-shard ranks
# over gloo, 4 tile-shard ranks), then the complete C5 render at N=1 with the current kernel.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run9}
mkdir -p "$OUT"
EXPLORE_OUT=r3b/run9 bash profiles/rehearse_n2.sh || exit 1
timeout -k 10 1000 python -u bench.py --workload c5 --no-cpu --no-pmc --no-diag --steps 10 --warmup 0 --progress \
    --json-out "$OUT/c5.json" > "$OUT/c5.log" 2>&1 || { tail -n 20 "$OUT/c5.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', round(d['value']), round(d['ms_per_step']), [round(x) for x in d['gather_ms_per_step']])"
