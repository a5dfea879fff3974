#!/bin/bash
# Round-2 GPU session 22: parity with four MSMs per launch at 2^18; prover batch; bench.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2z}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  run batch64_$rep 300 python bench.py --batch 64 --n 262144
  MSM_BATCH=2 run batch64_nm2_$rep 300 python bench.py --batch 64 --n 262144
done
run bench 300 python bench.py
