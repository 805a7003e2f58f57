#!/bin/bash
# Round 6: the complete C5 render at N = 1 on this round's library -- 10 progressive
# passes, 1024^2, 64^3 grid smoke, 50M photons per pass -- then rank 0 of an 8-GPU strong-scaling run of
# the same render and of C4's iteration 0, emulated on the one GPU (its packet share alone).
set -o pipefail
O=${1:-gpurun_out/r6/c5}; mkdir -p "$O"
export TMPDIR=/tmp
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', round(d['value']), round(d['ms_per_step'],1), [round(x) for x in d['gather_ms_per_step']])"; }
timeout -k 10 900 python -u bench.py --workload c5 --no-cpu --no-pmc --no-diag --steps 10 --warmup 0 --progress \
    --json-out "$O/c5.json" > "$O/c5.log" 2>&1 || { tail -n 20 "$O/c5.log"; exit 1; }
summ "$O/c5.json" c5_n1
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu --no-pmc --no-diag --steps 10 --warmup 0 --progress \
    --emulate-shard 0/8 --json-out "$O/c5_r0of8.json" > "$O/c5_r0of8.log" 2>&1 || { tail -n 20 "$O/c5_r0of8.log"; exit 1; }
summ "$O/c5_r0of8.json" c5_rank0_of_8
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu --no-pmc --no-diag --steps 1 --warmup 0 --progress \
    --emulate-shard 0/8 --json-out "$O/c4_r0of8.json" > "$O/c4_r0of8.log" 2>&1 || { tail -n 20 "$O/c4_r0of8.log"; exit 1; }
summ "$O/c4_r0of8.json" c4_rank0_of_8
