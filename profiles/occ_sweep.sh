#!/bin/bash
# Tile-kernel register budget sweep on the default C2 bench (no CPU leg / PMC passes).
# usage (repo root, via gpurun): [SCAN=0|1] profiles/occ_sweep.sh OUTDIR [occupancies...]
set -o pipefail
OUT=${1:-gpurun_out/occ}
shift || true
OCCS=("$@")
if [ ${#OCCS[@]} -eq 0 ]; then OCCS=(6 7 8); fi
mkdir -p "$OUT"
for o in "${OCCS[@]}"; do
  tag=s${SCAN:-0}o$o
  timeout -k 10 300 python -u bench.py --occupancy "$o" --scan-mode "${SCAN:-0}" --no-cpu --no-pmc --no-diag \
      --json-out "$OUT/$tag.json" > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -n 20 "$OUT/$tag.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', round(d['value']), round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
done
