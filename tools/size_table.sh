#!/bin/bash
# Bench lines at 2^16..2^20 on one GPU (pipelined throughput + single-MSM latency) -> one JSON per line.
#   bash tools/size_table.sh [out=gpurun_out/sizes.jsonl]
set -u
out=${1:-gpurun_out/sizes.jsonl}
mkdir -p gpurun_out
: > "$out"
for lg in 16 17 18 19 20; do
  timeout -k 10 120 python bench.py --n $((1 << lg)) --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/size_$lg.txt 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "ABORT 2^$lg rc=$rc" >&2; tail -5 gpurun_out/size_$lg.txt >&2; exit $rc; }
  grep '^{' gpurun_out/size_$lg.txt >> "$out"
  python3 -c "
import json
d = json.loads(open('gpurun_out/size_$lg.txt').read().split('\n')[-2] if False else [l for l in open('gpurun_out/size_$lg.txt') if l.startswith('{')][0])
print('2^$lg value %.4f ms/MSM  latency %.4f ms  c=%d K=%d  correct %s' % (d['value'], d['latency_ms'], d['config']['window_bits'], d['config']['run_length'], d['correct']))
" >&2
done
