#!/bin/bash
# Pipelined throughput (bench.py value, ms/MSM) over sizes x window widths: picks msm_best_window.
#   bash tools/window_sweep.sh "16 17 18 19 20" "13 14 15 16"
set -u
mkdir -p gpurun_out
for lg in $1; do
  for c in $2; do
    n=$((1 << lg))
    timeout -k 10 120 python bench.py --n $n --window $c --steps 30 --warmup 6 --no-cpu-baseline \
      > gpurun_out/ws_${lg}_${c}.txt 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "ABORT 2^$lg c=$c rc=$rc" >&2; tail -5 gpurun_out/ws_${lg}_${c}.txt >&2; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/ws_${lg}_${c}.txt'):
    if l.startswith('{'):
        d = json.loads(l); p = d['phases_ms']
        print('2^$lg c=$c value %.4f lat %.4f dev %.4f acc %.4f red %.4f fix %.4f K %d' % (d['value'], d['latency_ms'],
              p['device_total'], p['accumulate'], p['bucket_reduce_1'] + p['bucket_reduce_2'], p['fixup'], d['config']['run_length']))
" >&2
  done
done
