#!/bin/bash
# Round-2 GPU session 37: staged host uploads + two-phase host launches (sort starts on the
# scalars while the points upload): host-path GPU tests, e2e A/B (previous library, pack threads).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2aq}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gputests 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_js.py tests/test_gpu_msm.py -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  run new20_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_PACK_THREADS=16 run t16_20_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_PACK_THREADS=12 run t12_20_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_AMD_LIB=$L/libmsm_old.so run old20_$rep 120 python tools/e2e_probe.py --runs 8
done
run new19 120 python tools/e2e_probe.py --runs 8 --n 524288
MSM_PACK_THREADS=16 run t16_19 120 python tools/e2e_probe.py --runs 8 --n 524288
MSM_AMD_LIB=$L/libmsm_old.so run old19 120 python tools/e2e_probe.py --runs 8 --n 524288
MSM_PACK_THREADS=16 run prof 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_e2e -o run -- python3 tools/e2e_probe.py --runs 6
