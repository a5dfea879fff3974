#!/bin/bash
# Round-2 GPU session 11: 20- vs 50-step bench on one box; run length and batch at 2^17 / 2^18.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2m}
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 1 "gpurun_out/${TAG}_$name.txt" | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for rep in 1 2; do
  run b20_$rep 200 python bench.py --no-cpu-baseline
  run b50_$rep 200 python bench.py --no-cpu-baseline --steps 50 --warmup 20
done
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  run k16_$rep 120 $B --n 131072
  run k32_$rep 120 $B --n 131072 --run-length 32
  run k64_$rep 120 $B --n 131072 --run-length 64
  MSM_BATCH=4 run nm4_$rep 120 $B --n 131072
  MSM_BATCH=4 run nm4k32_$rep 120 $B --n 131072 --run-length 32
  run k32_18_$rep 120 $B --n 262144
  run k64_18_$rep 120 $B --n 262144 --run-length 64
  MSM_BATCH=4 run nm4_18_$rep 120 $B --n 262144
done
