#!/bin/bash
# Round-2 GPU session: parity tests, bench variants, ISA rates.  Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2c}
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/${TAG}_$name.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run bench 300 python bench.py
run bench_overlap 300 env MSM_ACC_OVERLAP=1 python bench.py --no-extras --no-cpu-baseline
run bench50 300 python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline
run batch64 300 python bench.py --batch 64 --n 262144
run isa_rates 120 tools/ubench/isa_rates
