#!/bin/bash
# Round-2 GPU session 34: host-input uploads from a helper thread (device-ordered on the slot's
# previous launch): host-path GPU tests, e2e probe, e2e timeline with copies.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2am}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 gpurun_out/${TAG}_$name.txt | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run e2e_1 120 python tools/e2e_probe.py --runs 8
run e2e_2 120 python tools/e2e_probe.py --runs 8
run e2e19 120 python tools/e2e_probe.py --runs 8 --n 524288
run prof 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_e2e -o run -- python3 tools/e2e_probe.py --runs 6
