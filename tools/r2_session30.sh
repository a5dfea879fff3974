#!/bin/bash
# Round-2 GPU session 30: kernel timeline of pipelined calls (two slots) at 2^20 and 2^17.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ah}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run probe20 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_probe20 -o run -- python3 tools/pipeline_probe.py --steps 20 --calls 4
run probe17 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_probe17 -o run -- python3 tools/pipeline_probe.py --steps 20 --calls 4 --n 131072
