#!/bin/bash
# Round-2 GPU session 28: JS flat-input test + node e2e; run length 96/128 at 2^20 (one round).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2af}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|passed.*\|failed.*\|"node_e2e_ms": [0-9.]*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run js 300 python -u -m pytest tests/test_gpu_js.py -m gpu -q --timeout 200 --timeout-method thread
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  run k64_$rep 120 $B
  run k96_$rep 120 $B --run-length 96
  run k128_$rep 120 $B --run-length 128
done
run bench 300 python bench.py --no-cpu-baseline
