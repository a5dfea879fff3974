#!/bin/bash
# Round-2 GPU session 4 (fresh container): parity tests, default bench, 50-step bench, prover batch,
# microbenchmarks, rocprof stats of the bench.  Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2f}
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
lscpu > gpurun_out/${TAG}_lscpu.txt 2>&1 || true
run pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run bench 300 python bench.py
run bench50 300 python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline
run batch64 300 python bench.py --batch 64 --n 262144
run isa_rates 120 tools/ubench/isa_rates
run fmul 120 tools/ubench/fmul_bench
run h2d 300 tools/ubench/h2d_bench 160
export TMPDIR=/tmp
run bench_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bench_prof -- python3 bench.py --no-cpu-baseline --no-extras
