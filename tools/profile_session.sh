#!/bin/bash
# GPU tests, bench, rocprofv3 kernel-trace summaries of bench runs (pipelined, and single-slot for
# clean per-kernel durations), and the PMC passes.  Usage: bash tools/profile_session.sh <tag>
set -u
tag=${1:-r1}
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
run bench 300 python bench.py
export TMPDIR=/tmp
run kstats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/kstats_$tag" -o run -- python bench.py --no-cpu-baseline
MSM_SLOTS=1 run kstats1 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/kstats1_$tag" -o run -- python bench.py --no-cpu-baseline
if [ "${PMC:-1}" = "1" ]; then
  run pmc 900 bash tools/profile_pmc.sh "$tag"
  python tools/pmc_summary.py "gpurun_out/pmc_$tag" 1048576 "gpurun_out/pmc_$tag/traffic.json" > "gpurun_out/pmc_$tag/summary.json" 2>&1 || true
fi
