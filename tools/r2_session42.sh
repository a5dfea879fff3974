#!/bin/bash
# Round-2 GPU session 42: host-input runs start the last launch's sort on its scalars while its
# points upload (MSM_HOST_SORT_EARLY=0: off): host-path GPU tests, e2e A/B at 2^20 / 2^19.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2az}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gputests 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_js.py tests/test_gpu_random_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  run on20_$rep 120 python tools/e2e_probe.py --runs 10
  MSM_HOST_SORT_EARLY=0 run off20_$rep 120 python tools/e2e_probe.py --runs 10
  run on19_$rep 120 python tools/e2e_probe.py --runs 10 --n 524288
  MSM_HOST_SORT_EARLY=0 run off19_$rep 120 python tools/e2e_probe.py --runs 10 --n 524288
done
