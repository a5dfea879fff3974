#!/bin/bash
# Round-2 final measurement session (second pass, after the nontemporal-store and merged-copy changes):
# prover batch), rocprofv3 summaries (default command; single stream 2^20) and PMC passes, e2e.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2final2}
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
lscpu > gpurun_out/${TAG}_lscpu.txt 2>&1 || true
run pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run bench 300 python bench.py
run bench_b 300 python bench.py --no-cpu-baseline
run bench50 300 python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline
for lg in 16 17 18 19; do
  run size$lg 120 python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline --n $((1 << lg))
  run size${lg}_k20 120 python bench.py --no-extras --no-cpu-baseline --n $((1 << lg))
done
run batch64 300 python bench.py --batch 64 --n 262144
run e2e 120 python tools/e2e_probe.py --runs 8
run kstats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kstats -o run -- python3 bench.py
MSM_SLOTS=1 run kstats1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kstats1 -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 4 --serial-min-s 0
