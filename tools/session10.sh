#!/bin/bash
set -u
mkdir -p gpurun_out
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 3 "gpurun_out/$name.txt" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -m pytest tests -m gpu -q -x --timeout 600
run sweep 400 python tools/sweep.py --libs libmsm_base.so,libmsm.so,libmsm_base.so,libmsm.so --windows 16 --runs 64 --steps 30
