#!/bin/bash
# Round-2 GPU session 19: k_bucket_reduce_2 workgroup size A/B (512 default vs 256/128/64 threads).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r2v}
L=$PWD/webgpu-msm_amd/msm_amd/_lib
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|passed.*\|failed.*' gpurun_out/${TAG}_$name.txt | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MSM_AMD_LIB=$L/libmsm_r2t64.so run t64 600 python -u -m pytest tests/test_gpu_msm.py -m gpu -x -q --timeout 300 --timeout-method thread -k "windows or survey or pipelined or skew or giant"
B="python bench.py --steps 50 --warmup 20 --no-extras --no-cpu-baseline"
for rep in 1 2; do
  for lg in 16 17 20; do
    run base_${lg}_$rep 120 $B --n $((1 << lg))
    for v in 64 128 256; do
      MSM_AMD_LIB=$L/libmsm_r2t$v.so run t${v}_${lg}_$rep 120 $B --n $((1 << lg))
    done
  done
done
for v in 64 128; do
  MSM_AMD_LIB=$L/libmsm_r2t$v.so MSM_SLOTS=1 run ks${v}_17 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ks${v}_17 -o run -- python3 bench.py --no-extras --no-cpu-baseline --n 131072 --steps 20 --warmup 4 --serial-min-s 0
done
