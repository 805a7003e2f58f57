set -o pipefail
mkdir -p gpurun_out/sweep3
run() {
  timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-diag "$@" > gpurun_out/sweep3/last.log 2>&1 || { tail -n 20 gpurun_out/sweep3/last.log; exit 1; }
  echo "$* -> $(grep '^{' gpurun_out/sweep3/last.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],1), "ms/step")')"
}
run --split 4
run --split 2
run --split 1
run --split 8 --loose-cos 1
run --split 4 --loose-cos 1
run --split 2 --loose-cos 1
run --split 8 --loose-cos 9000
run --split 4 --sort-segments 0
