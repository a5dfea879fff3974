#!/bin/bash
# Round-2 GPU session 47: odd slice count once more, padding MSMs no longer upload
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2be}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MSM_HOST_ODD=1 run gputests 600 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  run on20_$rep 120 python tools/e2e_probe.py --runs 10
  MSM_HOST_ODD=1 run odd20_$rep 120 python tools/e2e_probe.py --runs 10
  run on19_$rep 120 python tools/e2e_probe.py --runs 10 --n 524288
  MSM_HOST_ODD=1 run odd19_$rep 120 python tools/e2e_probe.py --runs 10 --n 524288
done
