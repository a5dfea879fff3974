#!/bin/bash
# Round-2 GPU session 16: launches in flight (slots) 1/2/3 at 2^16..2^18 and 2^20, 20 and 50 steps.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2s}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$name.txt | tail -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for rep in 1 2; do
  for lg in 16 17 18 20; do
    for sl in 1 2 3; do
      MSM_SLOTS=$sl run s${sl}_${lg}_k20_$rep 120 python bench.py --no-extras --no-cpu-baseline --n $((1 << lg))
      MSM_SLOTS=$sl run s${sl}_${lg}_k50_$rep 120 python bench.py --no-extras --no-cpu-baseline --n $((1 << lg)) --steps 50 --warmup 20
    done
  done
done
