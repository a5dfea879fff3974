#!/bin/bash
# Round-2 GPU session 33: nontemporal record stores in k_prepare_points (size-gated): full GPU
# tests, then A/B against MSM_PP_NT=0 at 2^20 / 2^19 and the 64 x 2^18 batch.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ak}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$name.txt | head -1) $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-120)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  run nt20_$rep 120 $B
  MSM_PP_NT=0 run t20_$rep 120 $B
  run nt19_$rep 120 $B --n 524288
  MSM_PP_NT=0 run t19_$rep 120 $B --n 524288
done
run ntb 200 python bench.py --batch 64 --n 262144 --steps 3 --warmup 1 --no-extras --no-cpu-baseline
MSM_PP_NT=0 run tb 200 python bench.py --batch 64 --n 262144 --steps 3 --warmup 1 --no-extras --no-cpu-baseline
