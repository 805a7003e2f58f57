#!/bin/bash
# Round 5 (via gpurun): the multi-rank bench flow's film digest at N = 1, 2, 4 (packet shards with
# packet-class films; N > 1 as ranks sharing the one GPU over gloo): equal digests show the split
# changes no bit of the rendered film.
set -o pipefail
OUT=${1:-gpurun_out/r5/digest}
mkdir -p "$OUT"
export TMPDIR=/tmp
A="--steps 4 --warmup 1 --no-cpu --no-pmc --no-legs"
timeout -k 10 300 python -u bench.py $A --json-out "$OUT/n1.json" > "$OUT/n1.log" 2>&1 || { tail -n 20 "$OUT/n1.log"; exit 1; }
for n in 2 4; do
  timeout -k 10 300 python -u bench.py --gpus $n --dist-backend gloo --share-gpu $A --json-out "$OUT/n$n.json" \
      > "$OUT/n$n.log" 2>&1 || { tail -n 30 "$OUT/n$n.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys
for n in (1, 2, 4):
    d = json.load(open(f"{sys.argv[1]}/n{n}.json"))
    print("N", n, "digest", d["film_digest"], "value", round(d["value"]), "ms", round(d["ms_per_step"], 1))
PY
