#!/bin/bash
# Build the tile-kernel profiling ablations (BRE_ABLATE 2..5) as separate libraries; since round 6 they
# need profiles/r6/negative/ablation_switches_r6.patch applied to bre_gather.hip first
# and time each on the default C2 bench (results are NOT correct images: timing only).
# Build (here, CPU):  profiles/ablate.sh build
# Run (GPU box):      profiles/ablate.sh run OUTDIR [bench args]
set -o pipefail
HERE=$(cd "$(dirname "$0")/.." && pwd)
CS=$HERE/beam-radiance-estimate-pbrt_amd/csrc
AB=$CS/build/ablate
if [ "$1" = build ]; then
  mkdir -p "$AB"
  FLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -I$CS -I$HERE/include"
  for k in 1 2 3 4; do
    /opt/rocm/bin/hipcc $FLAGS -DBRE_ABLATE=$k -c "$CS/bre_gather.hip" -o "$AB/bre_gather_$k.o" || exit 1
    objs=$(ls "$CS"/build/*.o | grep -v bre_gather.o)
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$AB/libbre_ablate$k.so" "$AB/bre_gather_$k.o" $objs || exit 1
  done
  echo built
  exit 0
fi
OUT=${2:-gpurun_out/ablate}
shift 2
mkdir -p "$OUT"
for k in 0 1 2 3 4; do
  lib=$CS/../libbre.so
  [ "$k" != 0 ] && lib=$AB/libbre_ablate$k.so
  BRE_LIBRARY=$lib timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/a$k.json" "$@" \
      > "$OUT/a$k.log" 2>&1 || { echo "ablation $k failed"; tail -n 20 "$OUT/a$k.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/a$k.json'));print('ablate $k', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
done
