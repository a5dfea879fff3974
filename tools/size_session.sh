#!/bin/bash
# Per-size study: bench (pipelined) at 2^16..2^20 and a window sweep at 2^17/2^18.
set -u
mkdir -p gpurun_out
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  grep -v amdgpu.ids "gpurun_out/$name.txt" | tail -n 8 | cut -c1-400 >&2
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
for lg in 16 17 18 19; do
  run bench_$lg 300 python bench.py --n $((1<<lg)) --steps 30 --warmup 5 --no-cpu-baseline
done
run sweep17 300 python tools/sweep.py --logn 17 --windows 11,12,13,14,15,16 --runs 64 --steps 20
run sweep18 300 python tools/sweep.py --logn 18 --windows 12,13,14,15,16 --runs 64 --steps 20
