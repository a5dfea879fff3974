#!/bin/bash
# Round-2 GPU session 7: per-kernel single-stream profiles of the pipelined plan at 2^16..2^19
# (small shards of the multi-GPU config) and of the 2^18 prover batch; the reworked bench line.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2i}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 1 "gpurun_out/${TAG}_$name.txt" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for lg in 16 17 18 19; do
  MSM_SLOTS=1 run ks$lg 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ks$lg -o run -- python3 bench.py --no-extras --no-cpu-baseline --n $((1 << lg))
done
MSM_SLOTS=1 run ksb 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ksb -o run -- python3 bench.py --batch 16 --n 262144 --steps 4 --warmup 1
run bench 300 python bench.py
run bench17 300 python bench.py --n 131072 --no-extras --no-cpu-baseline
run batch64 300 python bench.py --batch 64 --n 262144
