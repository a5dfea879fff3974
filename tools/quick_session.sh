#!/bin/bash
# GPU tests + smoke + bench + kernel-trace stats (no PMC). Stops at the first crash/timeout.
#   bash tools/quick_session.sh <tag>
set -u
tag=${1:-r1}
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 6 "gpurun_out/$name.txt" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
export TMPDIR=/tmp
run kstats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/kstats_$tag" -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
