#!/bin/bash
# Pipelined throughput for bucket-reduce chunk length L (MSM_RED_L) per size, auto window.
#   bash tools/l_sweep.sh "16 17 18 19 20" "4 8" [rounds]
set -u
mkdir -p gpurun_out
for r in $(seq 1 "${3:-1}"); do
for lg in $1; do
  for L in $2; do
    MSM_RED_L=$L timeout -k 10 120 python bench.py --n $((1 << lg)) --steps 30 --warmup 6 --no-cpu-baseline \
      > gpurun_out/ls_${lg}_${L}.txt 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "ABORT 2^$lg L=$L rc=$rc" >&2; tail -5 gpurun_out/ls_${lg}_${L}.txt >&2; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/ls_${lg}_${L}.txt'):
    if l.startswith('{'):
        d = json.loads(l); p = d['phases_ms']
        print('r$r 2^$lg L=$L c=%d value %.4f lat %.4f red1 %.4f red2 %.4f ok %s' % (d['config']['window_bits'], d['value'], d['latency_ms'], p['bucket_reduce_1'], p['bucket_reduce_2'], d['correct']))
" >&2
  done
done
done
