#!/bin/bash
# Pipelined bench value per environment setting and size (interleaved rounds).
#   bash tools/env_ab.sh "MSM_SLOTS=2 MSM_SLOTS=3" "17 20" [rounds]
set -u
mkdir -p gpurun_out
for r in $(seq 1 "${3:-1}"); do
for lg in $2; do
  for e in $1; do
    env "$e" timeout -k 10 120 python bench.py --n $((1 << lg)) --steps 40 --warmup 8 --no-cpu-baseline \
      > gpurun_out/eab.txt 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "ABORT $e 2^$lg rc=$rc" >&2; tail -5 gpurun_out/eab.txt >&2; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/eab.txt'):
    if l.startswith('{'):
        d = json.loads(l)
        print('r$r 2^$lg %-14s value %.4f lat %.4f ok %s' % ('$e', d['value'], d['latency_ms'], d['correct']))
" >&2
  done
done
done
