#!/bin/bash
# Round-2 GPU session 24: pipelined window width re-check at 2^16..2^19 with the current plan
# (4 MSMs per launch up to 2^18, two launches in flight, wave-fitted reduction chunks).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ab}
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
  for w in 12 13 14; do run w${w}_16_$rep 120 $B --n 65536 --window $w; done
  for w in 13 14 15; do run w${w}_17_$rep 120 $B --n 131072 --window $w; done
  for w in 14 15 16; do run w${w}_18_$rep 120 $B --n 262144 --window $w; done
  for w in 14 15 16; do run w${w}_19_$rep 120 $B --n 524288 --window $w; done
done
