#!/bin/bash
# One GPU session: GPU tests, smoke, bench.  Stops at the first crash/timeout (not at plain
# test failures, exit 1).  Usage: bash tools/gpu_session.sh [pytest-args...]
set -u
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 25 "gpurun_out/$name.txt" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
run pytest_gpu 1200 python -m pytest tests -m gpu -q -x --timeout 600 "$@"
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 10 --warmup 2
