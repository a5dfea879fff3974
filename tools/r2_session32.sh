#!/bin/bash
# Round-2 GPU session 32: k_prepare_points variants (nontemporal load/store, 5 waves/SIMD with
# spills, 128-thread blocks): parity subset, single-stream kernel times, bench A/B at 2^20 / 2^17.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2aj}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
T="python -u -m pytest tests/test_gpu_msm.py -m gpu -q -x --timeout 120 --timeout-method thread -k survey"
export TMPDIR=/tmp
for v in nt3 w5 t128; do
  MSM_AMD_LIB=$L/libmsm_$v.so run t_$v 300 $T
done
for v in base nt1 nt2 nt3 w5 t128; do
  lib=$L/libmsm_$v.so; [ $v = base ] && lib=$L/libmsm.so
  MSM_AMD_LIB=$lib MSM_SLOTS=1 run prof_$v 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$v -o run -- python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline
done
for rep in 1 2; do
  for v in base nt1 nt2 nt3 w5 t128; do
    lib=$L/libmsm_$v.so; [ $v = base ] && lib=$L/libmsm.so
    MSM_AMD_LIB=$lib run ${v}20_$rep 120 $B
    MSM_AMD_LIB=$lib run ${v}17_$rep 120 $B --n 131072
  done
done
