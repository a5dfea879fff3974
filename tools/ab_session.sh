#!/bin/bash
# A/B session: ISA issue rates + library-variant sweep.  Stops at the first crash/timeout.
#   bash tools/ab_session.sh <libs> [extra sweep args]
set -u
mkdir -p gpurun_out
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 20 "gpurun_out/$name.txt" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
libs=$1; shift
if [ -x tools/ubench/isa_rates ] && [ "${ISA_RATES:-0}" = 1 ]; then run isa_rates 120 tools/ubench/isa_rates; fi
run sweep 600 python tools/sweep.py --libs "$libs" --windows 16 --runs 64 --steps 30 "$@"
