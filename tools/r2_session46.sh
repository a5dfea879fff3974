#!/bin/bash
# Round-2 GPU session 46: padding MSMs of a short last launch upload nothing (they read the last
# real MSM's wire buffers): GPU tests, e2e A/B at n = 10^6 (7 slices: a short last launch) and 2^20.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2bd}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gputests 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_js.py tests/test_gpu_random_sweep.py tests/test_gpu_msm.py -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  run new1e6_$rep 120 python tools/e2e_probe.py --runs 8 --n 1000000
  MSM_AMD_LIB=$L/libmsm_old.so run old1e6_$rep 120 python tools/e2e_probe.py --runs 8 --n 1000000
  run new20_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_AMD_LIB=$L/libmsm_old.so run old20_$rep 120 python tools/e2e_probe.py --runs 8
done
