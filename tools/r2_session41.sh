#!/bin/bash
# Round-2 GPU session 41: field-multiply products as v_mad_i64_i32 row blocks (MSM_MAD_ASM=1)
# vs the compiler's v_mad_u64_u32 (libmsm_u64.so): full GPU tests, bench A/B at 2^20 / 2^17 /
# batch, single-stream kernel times of both.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2av}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|[0-9]* passed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; tail -5 gpurun_out/${TAG}_$name.txt; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  run asm20_$rep 120 $B
  MSM_AMD_LIB=$L/libmsm_u64.so run u64_20_$rep 120 $B
  run asm17_$rep 120 $B --n 131072
  MSM_AMD_LIB=$L/libmsm_u64.so run u64_17_$rep 120 $B --n 131072
done
run asmb 200 python bench.py --batch 64 --n 262144 --steps 3 --warmup 1 --no-extras --no-cpu-baseline
MSM_AMD_LIB=$L/libmsm_u64.so run u64b 200 python bench.py --batch 64 --n 262144 --steps 3 --warmup 1 --no-extras --no-cpu-baseline
MSM_SLOTS=1 run kasm 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kasm -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 4 --serial-min-s 0
MSM_SLOTS=1 MSM_AMD_LIB=$L/libmsm_u64.so run ku64 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ku64 -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 4 --serial-min-s 0
