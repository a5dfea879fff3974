#!/bin/bash
# GPU tests, then window sweeps per size (non-pipelined device time) and pipelined bench per size.
set -u
mkdir -p gpurun_out
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  grep -v amdgpu.ids "gpurun_out/$name.txt" | tail -n 4 | cut -c1-300 >&2
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || run pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
for lg in ${SIZES:-16 17 18 19 20}; do
  run tsweep_$lg 300 python tools/sweep.py --logn $lg --windows ${WINDOWS:-12,13,14,15,16,17} --runs 0 --steps 20
done
for lg in ${SIZES:-16 17 18 19 20}; do
  run tbench_$lg 300 python bench.py --n $((1<<lg)) --steps 40 --warmup 8 --no-cpu-baseline
done
