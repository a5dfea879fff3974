#!/bin/bash
# Round-2 GPU session 17: parity with two slots; e2e (host split) two vs three slots; bench lines.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2t}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"e2e_ms": \[[^]]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | tail -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  run e2e_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_SLOTS=3 run e2e_s3_$rep 120 python tools/e2e_probe.py --runs 8
done
run bench 300 python bench.py
run batch64 300 python bench.py --batch 64 --n 262144
MSM_SLOTS=3 run batch64_s3 300 python bench.py --batch 64 --n 262144
rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
MSM_SLOTS=1 bash tools/profile_pmc.sh ${TAG}_20 > gpurun_out/${TAG}_pmc.log 2>&1 && echo "pmc ok" || echo "pmc rc=$?"
