# parameter sweep of the auto gather on C2 (2 timed iterations each)
set -o pipefail
mkdir -p gpurun_out/sweep2
run() {
  timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-diag "$@" > gpurun_out/sweep2/last.log 2>&1 || { tail -n 20 gpurun_out/sweep2/last.log; exit 1; }
  echo "$* -> $(grep '^{' gpurun_out/sweep2/last.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],1), "ms/step")')"
}
run
run --loose-cos 9900
run --loose-cos 9700
run --loose-cos 9000
run --loose-cos 1
run --tile-leaf 16
run --tile-leaf 64
run --split 8
run --split 32
