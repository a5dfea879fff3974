#!/bin/bash
# Round-2 GPU session 29: timing-only probe -- does k_accumulate run faster at 5 waves per SIMD?
# libmsm_exp5.so keeps 32 head slots in LDS (WRONG results; timing only) and caps VGPRs at 96.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ag}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for lib in libmsm libmsm_exp5; do
  MSM_AMD_LIB=$L/$lib.so MSM_SLOTS=1 run ks_$lib 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ks_$lib -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 4 --serial-min-s 0
done
