#!/bin/bash
# A/B session: GPU tests on the default build, then bench for each library variant given.
# Usage: bash tools/ab_session.sh libA.so libB.so ...   (paths relative to webgpu-msm_amd/msm_amd/_lib)
set -u
mkdir -p gpurun_out
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 15 "gpurun_out/$name.txt" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -m pytest tests -m gpu -q -x --timeout 600
for v in "$@"; do
  MSM_AMD_LIB=$PWD/webgpu-msm_amd/msm_amd/_lib/$v run bench_$v 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
done
