#!/bin/bash
# Round-2 GPU session 48: up to eight MSMs per launch (MSM_MAX_BATCH 8): MSM_BATCH=8 / 6 vs the
# default four at 2^16 / 2^17 (the 8-GPU shard) and the 64 x 2^18 batch; GPU tests with MSM_BATCH=8.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2bg}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; tail -5 gpurun_out/${TAG}_$name.txt; exit $rc; fi
  return 0
}
B="python bench.py --steps 48 --warmup 16 --no-extras --no-cpu-baseline"
MSM_BATCH=8 run t8 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_random_sweep.py tests/test_gpu_paths.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not serial_flag"
for rep in 1 2 3; do
  run d17_$rep 120 $B --n 131072
  MSM_BATCH=8 run b8_17_$rep 120 $B --n 131072
  MSM_BATCH=8 MSM_RED_L=20 run b8L20_17_$rep 120 $B --n 131072
  run d16_$rep 120 $B --n 65536
  MSM_BATCH=8 run b8_16_$rep 120 $B --n 65536
done
run db 200 python bench.py --batch 64 --n 262144 --steps 3 --warmup 1 --no-extras --no-cpu-baseline
MSM_BATCH=8 run b8b 200 python bench.py --batch 64 --n 262144 --steps 3 --warmup 1 --no-extras --no-cpu-baseline
