#!/bin/bash
# Round-2 GPU session 36: staged host uploads (pinned ring, x|y|t compaction, pack pool): GPU
# tests, e2e A/B against the previous library and MSM_STAGE=0, pack-thread counts.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ap}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2; do
  run new20_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_AMD_LIB=$L/libmsm_old.so run old20_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_STAGE=0 run nostage20_$rep 120 python tools/e2e_probe.py --runs 8
  run new19_$rep 120 python tools/e2e_probe.py --runs 8 --n 524288
  MSM_AMD_LIB=$L/libmsm_old.so run old19_$rep 120 python tools/e2e_probe.py --runs 8 --n 524288
done
for t in 4 16; do
  MSM_PACK_THREADS=$t run th${t}_20 120 python tools/e2e_probe.py --runs 8
done
run prof 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_e2e -o run -- python3 tools/e2e_probe.py --runs 6
