#!/bin/bash
# Round-2 GPU session 12: why 20 timed steps read slower than 50 -- consecutive calls and the
# length of the untimed serial pass before the timed region.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2n}
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
run probe 200 python tools/pipeline_probe.py --steps 20 --calls 8
for rep in 1 2; do
  run s8_$rep 200 python bench.py --no-cpu-baseline --no-extras
  run s32_$rep 200 python bench.py --no-cpu-baseline --no-extras --serial-msms 32
  run s64_$rep 200 python bench.py --no-cpu-baseline --no-extras --serial-msms 64
  run s8x50_$rep 200 python bench.py --no-cpu-baseline --no-extras --steps 50 --warmup 20
done
