#!/bin/bash
# GPU tests then an A/B sweep (libs as $1).  Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 12 "gpurun_out/$name.txt" >&2
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
run sweep 600 python tools/sweep.py --libs "$1" --windows 16 --runs 64 --steps 30
