#!/bin/bash
# Round-2 GPU session 6: pipeline fill/drain probe (kernel trace of K=20 and K=50 calls) and the
# single-stream rocprofv3 summary the bench's roofline kernel_ms must agree with.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2h}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 2 "gpurun_out/${TAG}_$name.txt" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run probe 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_probe -o run -- python3 tools/pipeline_probe.py --steps 20 --calls 3
run probe50 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_probe50 -o run -- python3 tools/pipeline_probe.py --steps 50 --calls 2
MSM_SLOTS=1 run kstats1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kstats1 -o run -- python3 bench.py --no-extras --no-cpu-baseline
