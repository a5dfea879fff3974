#!/bin/bash
# Round-2 GPU session 13: parity with four-MSM launches (L = 17 at 2^17), A/B vs two, e2e, bench.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2o}
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
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  for lg in 16 17; do
    run nm4_${lg}_$rep 120 $B --n $((1 << lg))
    MSM_BATCH=2 run nm2_${lg}_$rep 120 $B --n $((1 << lg))
  done
done
run e2e 120 python tools/e2e_probe.py --runs 8
run bench 300 python bench.py
run bench17 300 python bench.py --n 131072 --no-cpu-baseline
