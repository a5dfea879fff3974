#!/bin/bash
# Round-2 GPU session 2: single-graph timed launches, multirank tests, e2e probes, timeline.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2d}
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "gpurun_out/${TAG}_$name.txt" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run bench 300 python bench.py
run bench50 300 python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline
run slots1 300 env MSM_SLOTS=1 python bench.py --no-extras --no-cpu-baseline
run e2e 120 python tools/e2e_probe.py
run e2e_pin 120 env MSM_H2D_PIN=1 python tools/e2e_probe.py
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run e2e_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r2d_e2e_trace -- python3 tools/e2e_probe.py --runs 3
