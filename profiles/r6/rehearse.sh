#!/bin/bash
# Round 6: the multi-rank bench flow rehearsed on the one-GPU box -- 1, 2 and 4 ranks
# (torch.distributed.run, every rank on cuda:0, collectives over gloo), packet shards with packet-class
# films.  (a) --workload c4-1m (the 2K tiled film at 1M photons): the film digests of N = 1, 2, 4 must be
# equal; (b) the default C2 line at N = 2 with its config legs: each leg carries the live rank count, the
# per-rank gather times and its own film digest, to be compared with the N = 1 legs.
set -o pipefail
O=${1:-gpurun_out/r6/rehearse}; mkdir -p "$O"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
dig() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
legs = {k: (v.get("ranks_live"), (v.get("film_digest") or {}).get("sha256"), [round(x, 1) for x in v.get("gather_ms_per_rank", [])])
        for k, v in (d.get("config_legs") or {}).items()}
print(sys.argv[2], "n_gpus", d["n_gpus"], "value", round(d["value"]), "ms/step", round(d["ms_per_step"], 1),
      "digest", (d.get("film_digest") or {}).get("sha256"), "legs", legs)
PY
}
for n in 1 2 4; do
  timeout -k 10 400 python -u bench.py --workload c4-1m --gpus $n --dist-backend gloo --share-gpu --steps 2 --warmup 1 \
      --no-cpu --no-pmc --no-diag --json-out "$O/c4_1m_n$n.json" > "$O/c4_1m_n$n.log" 2>&1 || { tail -n 30 "$O/c4_1m_n$n.log"; exit 1; }
  dig "$O/c4_1m_n$n.json" "c4-1m N=$n"
done
for n in 1 2; do
  timeout -k 10 600 python -u bench.py --gpus $n --dist-backend gloo --share-gpu --steps 2 --warmup 1 --no-cpu --no-pmc \
      --no-diag --json-out "$O/c2_legs_n$n.json" > "$O/c2_legs_n$n.log" 2>&1 || { tail -n 30 "$O/c2_legs_n$n.log"; exit 1; }
  dig "$O/c2_legs_n$n.json" "c2+legs N=$n"
done
