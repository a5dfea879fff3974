#!/bin/bash
# Round-2 GPU session 25: run length filling whole accumulation rounds (K = 36 at 2^17 / 2^18,
# 20 at 2^16) vs the previous power-of-two choice; parity; c = 16 at 2^19.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ac}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  run n16_$rep 120 $B --n 65536
  run o16_$rep 120 $B --n 65536 --run-length 16
  run n17_$rep 120 $B --n 131072
  run o17_$rep 120 $B --n 131072 --run-length 32
  run n18_$rep 120 $B --n 262144
  run o18_$rep 120 $B --n 262144 --run-length 64
  run n19_$rep 120 $B --n 524288
  run n20_$rep 120 $B
done
run batch64 300 python bench.py --batch 64 --n 262144
