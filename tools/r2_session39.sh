#!/bin/bash
# Round-2 GPU session 39: window width re-sweep at 2^16-2^18 and the 64 x 2^18 batch with the
# current plan (four MSMs per launch, wave-fitted reduction chunks).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2at}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  for c in 13 14 15 16; do run n17_c${c}_$rep 120 $B --n 131072 --window $c; done
  for c in 14 15 16; do run n18_c${c}_$rep 120 $B --n 262144 --window $c; done
  for c in 13 14 15; do run n16_c${c}_$rep 120 $B --n 65536 --window $c; done
done
for c in 14 15 16; do run b64_c$c 200 python bench.py --batch 64 --n 262144 --steps 3 --warmup 1 --no-extras --no-cpu-baseline --window $c; done
