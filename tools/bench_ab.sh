#!/bin/bash
# Pipelined bench value (ms/MSM) per library variant, interleaved rounds to gauge noise.
#   bash tools/bench_ab.sh libmsm.so,libmsm_x.so [rounds] [extra bench args]
set -u
mkdir -p gpurun_out
libs=$1; rounds=${2:-2}; shift 2 || shift $#
for r in $(seq 1 "$rounds"); do
  for lib in ${libs//,/ }; do
    MSM_AMD_LIB=$PWD/webgpu-msm_amd/msm_amd/_lib/$lib timeout -k 10 180 python bench.py --steps 40 --warmup 10 \
      --no-cpu-baseline "$@" > gpurun_out/bab_${lib%.so}_$r.txt 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "ABORT $lib rc=$rc" >&2; tail -5 gpurun_out/bab_${lib%.so}_$r.txt >&2; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/bab_${lib%.so}_$r.txt'):
    if l.startswith('{'):
        d = json.loads(l); p = d['phases_ms']
        print('r$r %-22s value %.4f lat %.4f red1 %.4f red2 %.4f ok %s' % ('$lib', d['value'], d['latency_ms'], p['bucket_reduce_1'], p['bucket_reduce_2'], d['correct']))
" >&2
  done
done
