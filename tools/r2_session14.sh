#!/bin/bash
# Round-2 GPU session 14: 20 vs 50 timed steps on one box (time-based hot serial pass), at 2^20 and
# at 2^17 with four or two MSMs per launch.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2q}
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
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  run b20_$rep 200 python bench.py --no-cpu-baseline
  run b50_$rep 200 python bench.py --no-cpu-baseline --steps 50 --warmup 20
  run s20_17_$rep 200 python bench.py --no-cpu-baseline --no-extras --n 131072
  run s50_17_$rep 200 python bench.py --no-cpu-baseline --no-extras --n 131072 --steps 50 --warmup 20
  MSM_BATCH=2 run s20_17nm2_$rep 200 python bench.py --no-cpu-baseline --no-extras --n 131072
done
