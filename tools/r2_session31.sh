#!/bin/bash
# Round-2 GPU session 31: stream priority experiment (slot 0 high) at 2^20 / 2^17 / batch.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ai}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2 3; do
  run d20_$rep 120 $B
  MSM_PRIO=1 run p20_$rep 120 $B
  run d17_$rep 120 $B --n 131072
  MSM_PRIO=1 run p17_$rep 120 $B --n 131072
done
run b20 120 python bench.py --no-extras --no-cpu-baseline
MSM_PRIO=1 run pb20 120 python bench.py --no-extras --no-cpu-baseline
