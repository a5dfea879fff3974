#!/bin/bash
# Round-2 GPU session 26: single-stream accumulate at 2^17 (four MSMs per launch), K = 36 vs 32.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2ad}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for k in 36 32 64; do
  MSM_SLOTS=1 run k$k 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_k$k -o run -- python3 bench.py --no-extras --no-cpu-baseline --n 131072 --steps 20 --warmup 4 --serial-min-s 0 --run-length $k
done
