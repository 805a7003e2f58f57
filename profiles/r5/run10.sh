#!/bin/bash
# Round 5 run 10 (via gpurun): k_roots with NREG = 4 frontier registers per lane at S = 256 -- root
# and split tests, sums bit for bit against the previous k_roots (variant base), kernel trace.
set -o pipefail
OUT=${1:-gpurun_out/r5/run10}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_split_gpu.py tests/test_root_shards_gpu.py tests/test_c2_production.py tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_film_determinism_gpu.py tests/test_pipeline_gpu.py > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
BRE_LIBRARY=beam-radiance-estimate-pbrt_amd/libbre.so timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_def.npz" c2 > "$OUT/bc_def.log" 2>&1 || exit 1
BRE_LIBRARY=$V/libbre_base.so timeout -k 10 200 python -u profiles/r5/bitcmp.py dump "$OUT/bc_base.npz" c2 > "$OUT/bc_base.log" 2>&1 || exit 1
python3 profiles/r5/bitcmp.py cmp "$OUT/bc_def.npz" "$OUT/bc_base.npz"; rm -f "$OUT"/*.npz
for S in 256 1024; do
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace$S" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --split $S --no-cpu --no-diag --no-pmc --no-legs > "$OUT/trace$S.log" 2>&1 || { tail -n 20 "$OUT/trace$S.log"; exit 1; }
grep -i "k_roots" "$OUT/trace$S/run_kernel_stats.csv" | cut -d, -f1-4
done
