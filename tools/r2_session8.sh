#!/bin/bash
# Round-2 GPU session 8: parity after fe_mul_2d + general-L bucket reduction; A/B of L = 9 vs 8
# (c = 15 pipelined sizes) and a single-stream profile at 2^17.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2j}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 1 "gpurun_out/${TAG}_$name.txt" | cut -c1-250
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  for lg in 17 18 20; do
    run new${lg}_$rep 120 $B --n $((1 << lg))
    MSM_RED_L=8 run l8_${lg}_$rep 120 $B --n $((1 << lg))
  done
done
MSM_SLOTS=1 run ks17 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ks17 -o run -- python3 bench.py --no-extras --no-cpu-baseline --n 131072
run batch64 300 python bench.py --batch 64 --n 262144
MSM_RED_L=8 run batch64_l8 300 python bench.py --batch 64 --n 262144
