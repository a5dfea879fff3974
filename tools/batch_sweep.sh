#!/bin/bash
# Pipelined throughput vs MSMs per launch (MSM_BATCH) per size and window.
#   bash tools/batch_sweep.sh "16:0 17:16" "1 2 3 4" [rounds]     (window 0 = auto)
set -u
mkdir -p gpurun_out
for r in $(seq 1 "${3:-1}"); do
for cfg in $1; do
  lg=${cfg%%:*}; c=${cfg##*:}
  for B in $2; do
    MSM_BATCH=$B timeout -k 10 120 python bench.py --n $((1 << lg)) --window $c --steps 40 --warmup 8 --no-cpu-baseline \
      > gpurun_out/bs_${lg}_${c}_${B}.txt 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "ABORT 2^$lg B=$B rc=$rc" >&2; tail -5 gpurun_out/bs_${lg}_${c}_${B}.txt >&2; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/bs_${lg}_${c}_${B}.txt'):
    if l.startswith('{'):
        d = json.loads(l)
        print('r$r 2^$lg B=$B c=%d K=%d value %.4f lat %.4f ok %s' % (d['config']['window_bits'], d['config']['run_length'], d['value'], d['latency_ms'], d['correct']))
" >&2
  done
done
done
