#!/bin/bash
# Round-2 GPU session 40: reduction chunk length L (MSM_RED_L) at 2^17 / 2^18 (four MSMs per
# launch) and 2^20 (two): is one wave per SIMD still the best fit?
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2au}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  run n17_auto_$rep 120 $B --n 131072
  for L in 8 9 10 12; do MSM_RED_L=$L run n17_L${L}_$rep 120 $B --n 131072; done
  run n18_auto_$rep 120 $B --n 262144
  for L in 8 10 12; do MSM_RED_L=$L run n18_L${L}_$rep 120 $B --n 262144; done
  run n20_auto_$rep 120 $B
  for L in 8 12; do MSM_RED_L=$L run n20_L${L}_$rep 120 $B; done
done
