#!/bin/bash
# Round-2 GPU session 15: single-stream kernel profiles of the current plans (2^16/2^17 four MSMs per
# launch, 2^18 two) and pipelined rates on the same box.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2r}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 1 "gpurun_out/${TAG}_$name.txt" | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for lg in 16 17 18; do
  MSM_SLOTS=1 run ks$lg 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ks$lg -o run -- python3 bench.py --no-extras --no-cpu-baseline --n $((1 << lg)) --steps 40 --warmup 8
  run p$lg 120 python bench.py --no-extras --no-cpu-baseline --n $((1 << lg)) --steps 40 --warmup 8
done
