#!/bin/bash
# Round-2 GPU session 3: graph event nodes, fill/drain probe, rocprof of the bench.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2e}
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "gpurun_out/${TAG}_$name.txt" | cut -c1-1200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_msm.py -m gpu -q --timeout 300 --timeout-method thread
run bench 300 python bench.py --no-cpu-baseline
run bench50 300 python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline
export TMPDIR=/tmp
run probe_trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_probe -- python3 tools/pipeline_probe.py
run bench_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bench_prof -- python3 bench.py --no-cpu-baseline --no-extras
