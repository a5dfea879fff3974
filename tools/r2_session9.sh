#!/bin/bash
# Round-2 GPU session 9: split host-input MSM (slices overlap the upload): parity, e2e A/B.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2k}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 1 "gpurun_out/${TAG}_$name.txt" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_msm.py -m gpu -x -q --timeout 300 --timeout-method thread -k "host or survey or partial or reference_format"
for rep in 1 2; do
  run e2e_split_$rep 120 python tools/e2e_probe.py --runs 8
  MSM_HOST_SPLIT=0 run e2e_nosplit_$rep 120 python tools/e2e_probe.py --runs 8
done
run e2e_19 120 python tools/e2e_probe.py --runs 8 --n 524288
MSM_HOST_SPLIT=0 run e2e_19_nosplit 120 python tools/e2e_probe.py --runs 8 --n 524288
run e2e_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_e2e_trace -o run -- python3 tools/e2e_probe.py --runs 3
run bench 300 python bench.py
