#!/bin/bash
# Full GPU session for a round: GPU tests, smoke, bench (with CPU baseline), rocprofv3 kernel-trace
# stats of a bench run, then the PMC passes.  Stops at the first crash/timeout.
#   bash tools/round_session.sh <tag>
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
run pytest_gpu 900 python -m pytest tests -m gpu -q -x --timeout 600
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 20 --warmup 3
export TMPDIR=/tmp
run kstats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/kstats_$tag" -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run pmc 900 bash tools/profile_pmc.sh "$tag"
python tools/pmc_summary.py "gpurun_out/pmc_$tag" 1048576 > "gpurun_out/pmc_$tag/summary.json" 2>&1 || true
