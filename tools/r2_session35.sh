#!/bin/bash
# Round-2 GPU session 35: host-input launches upload adjacent slices in one copy per array
# (A/B against the previous library): host-path GPU tests, e2e at 2^20 / 2^19.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2an}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gputests 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_js.py -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2; do
  run new20_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_AMD_LIB=$L/libmsm_old.so run old20_$rep 120 python tools/e2e_probe.py --runs 8
  run new19_$rep 120 python tools/e2e_probe.py --runs 8 --n 524288
  MSM_AMD_LIB=$L/libmsm_old.so run old19_$rep 120 python tools/e2e_probe.py --runs 8 --n 524288
done
