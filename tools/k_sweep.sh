#!/bin/bash
# Pipelined throughput over run length K (bench.py --run-length) for given sizes/windows.
#   bash tools/k_sweep.sh "17:15 18:15 19:15" "8 16 32 64"
set -u
mkdir -p gpurun_out
for cfg in $1; do
  lg=${cfg%%:*}; c=${cfg##*:}
  for k in $2; do
    timeout -k 10 120 python bench.py --n $((1 << lg)) --window $c --run-length $k --steps 30 --warmup 6 \
      --no-cpu-baseline > gpurun_out/ks_${lg}_${c}_${k}.txt 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "ABORT 2^$lg c=$c K=$k rc=$rc" >&2; tail -5 gpurun_out/ks_${lg}_${c}_${k}.txt >&2; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/ks_${lg}_${c}_${k}.txt'):
    if l.startswith('{'):
        d = json.loads(l); p = d['phases_ms']
        print('2^$lg c=$c K=$k value %.4f lat %.4f acc %.4f fix %.4f ok %s' % (d['value'], d['latency_ms'], p['accumulate'], p['fixup'], d['correct']))
" >&2
  done
done
