#!/bin/bash
# Pipelined throughput vs slots in flight, 2^16..2^20.
set -u
mkdir -p gpurun_out
for lg in ${SIZES:-16 17 18 19 20}; do
  for s in ${SLOTS:-2 3 4}; do
    echo "== lg=$lg slots=$s" >&2
    MSM_SLOTS=$s timeout -k 10 300 python bench.py --n $((1<<lg)) --steps 40 --warmup 8 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/slots_${lg}_${s}.txt 2>&1
    rc=$?
    python3 -c "import json,sys
for l in open('gpurun_out/slots_${lg}_${s}.txt'):
    if l.startswith('{'):
        d=json.loads(l); print('lg=$lg slots=$s value', d['value'], 'lat', d['latency_ms'], 'c', d['config']['window_bits'], 'ok', d['correct'])" >&2
    if [ $rc -ne 0 ]; then echo "ABORT rc=$rc" >&2; tail -5 gpurun_out/slots_${lg}_${s}.txt >&2; exit $rc; fi
  done
done
