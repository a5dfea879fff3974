#!/bin/bash
# Round-2 GPU session 23: reduction chunk length L re-check per size (env override) with the
# current batch/slot plan.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2aa}
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
  run d20_$rep 120 $B
  for l in 8 10 12; do MSM_RED_L=$l run l${l}_20_$rep 120 $B; done
  run d18_$rep 120 $B --n 262144
  for l in 12 16 20; do MSM_RED_L=$l run l${l}_18_$rep 120 $B --n 262144; done
  run d16_$rep 120 $B --n 65536
  for l in 4 9 10; do MSM_RED_L=$l run l${l}_16_$rep 120 $B --n 65536; done
done
