#!/bin/bash
# Round-2 GPU session 21: batch size re-check with two slots (2^18..2^20), per-size table.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2y}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  for lg in 18 19 20; do
    run d_${lg}_$rep 120 $B --n $((1 << lg))
    MSM_BATCH=1 run b1_${lg}_$rep 120 $B --n $((1 << lg))
    MSM_BATCH=4 run b4_${lg}_$rep 120 $B --n $((1 << lg))
  done
  run d_16_$rep 120 $B --n 65536
  run d_17_$rep 120 $B --n 131072
done
run js 300 python -u -m pytest tests/test_gpu_js.py -m gpu -q --timeout 200 --timeout-method thread
run node 300 python bench.py --no-cpu-baseline
